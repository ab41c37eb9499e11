source scripts/gpurun_lib.sh
run r9_debug.txt 300 python scripts/debug_variants.py
run r9_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r9_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
