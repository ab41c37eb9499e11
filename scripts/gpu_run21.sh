source scripts/gpurun_lib.sh
run r21_attn.txt 300 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k "attention or vit"
run r21_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r21_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r21_prof_vit.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit21 -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 3 --warmup 3
run r21_bench_r50.txt 300 python bench.py --steps 30 --warmup 10
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
