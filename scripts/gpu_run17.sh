source scripts/gpurun_lib.sh
run r17_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
PDT_BN_BLOCKS=512 run r17_bench_r50_512.txt 300 python bench.py --steps 30 --warmup 10
run r17_bench_r50_1024.txt 300 python bench.py --steps 30 --warmup 10
PDT_BN_BLOCKS=2048 run r17_bench_r50_2048.txt 300 python bench.py --steps 30 --warmup 10
run r17_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r17_gemm.txt 600 python scripts/bench_gemm.py --iters 10
exit 0
