source scripts/gpurun_lib.sh
run r68_pytest_gpu.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run r68_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()"
run r68_bench.txt 400 python bench.py
run r68_bench_b.txt 400 python bench.py
exit 0
