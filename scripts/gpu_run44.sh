source scripts/gpurun_lib.sh
run r44_tests.txt 600 python -u -m pytest tests/test_bn_fusion_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py tests/test_train_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "fusion or bottleneck or resnet50 or ddp or train"
run r44_bench_side.txt 400 python bench.py
PDT_WGRAD_STREAM=0 run r44_bench_noside.txt 400 python bench.py
run r44_bench_side2.txt 400 python bench.py
run r44_bench_side256.txt 400 python bench.py --batch 256
run r44_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_44 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
