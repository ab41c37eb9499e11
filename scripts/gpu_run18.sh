source scripts/gpurun_lib.sh
run r18_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r18_bench_r50a.txt 300 python bench.py --steps 30 --warmup 10
run r18_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
run r18_bench_r152.txt 400 python bench.py --model resnet152 --batch 512 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
