source scripts/gpurun_lib.sh
run r20_debug.txt 300 python scripts/debug_variants.py
run r20_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k "conv or gemm or f8 or linear or bottleneck or resnet"
run r20_gemm.txt 600 python scripts/bench_gemm.py --iters 10
exit 0
