source scripts/gpurun_lib.sh
run r15_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k "fp8 or f8 or version or vit"
run r15_prof_vit.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit15 -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 3 --warmup 3
run r15_prof_vit8.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit8_15 -o run --output-format csv -- python3 bench.py --model vit_b_16 --fp8 --steps 3 --warmup 3
run r15_bench_vit_fp8.txt 400 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
run r15_bench_r50a.txt 300 python bench.py --steps 30 --warmup 10
run r15_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
