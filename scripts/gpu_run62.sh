source scripts/gpurun_lib.sh
run r62_pytest_gpu.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run r62_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()"
run r62_bench.txt 400 python bench.py
run r62_bench_b.txt 400 python bench.py
exit 0
