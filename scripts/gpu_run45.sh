source scripts/gpurun_lib.sh
run r45_tests.txt 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_fusion_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "stream or conv or bottleneck or resnet50 or fusion"
run r45_bench_tune.txt 600 python bench.py --steps 10 --warmup 5
run r45_bench_tune256.txt 600 python bench.py --steps 10 --warmup 5 --batch 256
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r45_autotune_gfx950.json
run r45_bench_a.txt 400 python bench.py
run r45_bench_b.txt 400 python bench.py
run r45_bench_256.txt 400 python bench.py --batch 256
run r45_kbench.txt 600 python scripts/bench_kernels.py --iters 5
exit 0
