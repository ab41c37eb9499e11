source scripts/gpurun_lib.sh
run r8_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r8_bench_r50.txt 300 python bench.py --steps 30 --warmup 10
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
run r8_prof_vit.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit8 -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 3 --warmup 2
run r8_kbench.txt 400 python scripts/bench_kernels.py --iters 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
