source scripts/gpurun_lib.sh
run r25_attn.txt 300 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k "attention or vit"
run r25_bench_vit.txt 500 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r25_bench_vit8.txt 500 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
run r25_prof_vit8.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit8_25 -o run --output-format csv -- python3 bench.py --model vit_b_16 --fp8 --steps 3 --warmup 3
exit 0
