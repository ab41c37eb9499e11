source scripts/gpurun_lib.sh
run r6_tests.txt 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r6_kbench.txt 400 python scripts/bench_kernels.py --iters 5
run r6_bench_native.txt 300 python bench.py --backend native --steps 20 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
run r6_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native6 -o run --output-format csv -- python3 bench.py --backend native --steps 5 --warmup 3
exit 0
