source scripts/gpurun_lib.sh
run r19_debug.txt 300 python scripts/debug_variants.py
run r19_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r19_gemm.txt 600 python scripts/bench_gemm.py --iters 10
PDT_AUTOTUNE_CACHE=/tmp/t19.json run r19_bench_r50.txt 400 python bench.py --steps 30 --warmup 10
PDT_AUTOTUNE_CACHE=/tmp/t19.json run r19_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
PDT_AUTOTUNE_CACHE=/tmp/t19.json run r19_bench_vit8.txt 400 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
cp /tmp/t19.json gpurun_out/autotune_r19.json
exit 0
