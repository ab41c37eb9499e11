source scripts/gpurun_lib.sh
run r26_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r26_bench_r50a.txt 300 python bench.py --steps 30 --warmup 10
run r26_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
run r26_bench_vit.txt 500 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r26_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_26 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
