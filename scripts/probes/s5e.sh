source scripts/gpurun_lib.sh
run s5e_tests.txt 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread && \
run s5e_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()" && \
run s5e_bench.txt 400 python bench.py
