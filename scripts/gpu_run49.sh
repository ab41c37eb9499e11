source scripts/gpurun_lib.sh
run r49_tests.txt 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv_fwd_dgrad_wgrad or linear"
run r49_probe.txt 300 python scripts/probe_linear_wgrad.py
run r49_bench_a.txt 400 python bench.py
run r49_bench_256.txt 400 python bench.py --batch 256
run r49_bench_vit8.txt 400 python bench.py --model vit_b_16 --fp8 --steps 10 --warmup 5
run r49_kbench.txt 600 python scripts/bench_kernels.py --iters 5
exit 0
