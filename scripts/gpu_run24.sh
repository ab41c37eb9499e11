source scripts/gpurun_lib.sh
run r24_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r24_bench_r50a.txt 300 python bench.py --steps 30 --warmup 10
run r24_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
run r24_bench_vit8.txt 500 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
run r24_bench_r152.txt 500 python bench.py --model resnet152 --batch 512 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
