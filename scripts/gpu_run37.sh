source scripts/gpurun_lib.sh
run r37_tests.txt 600 python -u -m pytest tests/test_bn_fusion_gpu.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "fusion or bottleneck or resnet50" -s
run r37_bench_fuse.txt 400 python bench.py --steps 30 --warmup 10
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r37_autotune_gfx950.json
run r37_bench_fuse2.txt 300 python bench.py --steps 30 --warmup 10
PDT_FUSE_BN_BWD=0 run r37_bench_nofuse.txt 300 python bench.py --steps 30 --warmup 10
run r37_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_36 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
