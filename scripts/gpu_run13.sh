source scripts/gpurun_lib.sh
run r13_attn.txt 300 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k attention
run r13_debug.txt 300 python scripts/debug_variants.py
run r13_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r13_bench_r50.txt 300 python bench.py --steps 30 --warmup 10
run r13_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
run r13_bench_r152.txt 400 python bench.py --model resnet152 --batch 512 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
run r13_kbench.txt 400 python scripts/bench_kernels.py --iters 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
