source scripts/gpurun_lib.sh
run r12_debug.txt 300 python scripts/debug_variants.py
run r12_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r12_bench_r50.txt 300 python bench.py --steps 30 --warmup 10
run r12_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r12_bench_r152.txt 400 python bench.py --model resnet152 --batch 512 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
run r12_kbench.txt 400 python scripts/bench_kernels.py --iters 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
