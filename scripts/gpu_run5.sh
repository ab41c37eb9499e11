source scripts/gpurun_lib.sh
run r5_tests.txt 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r5_bench_native.txt 300 python bench.py --backend native --steps 20 --warmup 5
run r5_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native5 -o run --output-format csv -- python3 bench.py --backend native --steps 5 --warmup 3
exit 0
