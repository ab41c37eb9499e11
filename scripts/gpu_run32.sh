source scripts/gpurun_lib.sh
run r32_tests.txt 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv or stream or bottleneck or resnet50"
run r32_bench_r50a.txt 400 python bench.py --steps 30 --warmup 10
run r32_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r32_autotune_gfx950.json
run r32_kbench.txt 600 python scripts/bench_kernels.py --iters 5
exit 0
