source scripts/gpurun_lib.sh
run s4j_tests.txt 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread && \
run s4j_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()" && \
run s4j_bench.txt 400 python bench.py && \
run s4j_bench_r152.txt 600 python bench.py --model resnet152 --batch 2048 --steps 5 --warmup 3
