source scripts/gpurun_lib.sh
run r16_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r16_ddp.txt 300 python -m pytest tests/test_ddp_gpu.py -m gpu -q -p no:cacheprovider
run r16_bench_r50a.txt 300 python bench.py --steps 30 --warmup 10
run r16_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
run r16_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r16_bench_vit_fp8.txt 400 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
run r16_prof_vit.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit16 -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 3 --warmup 3
run r16_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_16 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
