source scripts/gpurun_lib.sh
run r27_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k "bn or bottleneck or resnet or conv_bn"
run r27_bench_r50a.txt 300 python bench.py --steps 30 --warmup 10
run r27_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
run r27_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_27 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
