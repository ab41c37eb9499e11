source scripts/gpurun_lib.sh
run r46_tests.txt 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv_fwd_dgrad_wgrad or linear"
run r46_bench_tune.txt 600 python bench.py --steps 10 --warmup 5
run r46_bench_tune256.txt 600 python bench.py --steps 10 --warmup 5 --batch 256
run r46_bench_tunevit.txt 600 python bench.py --model vit_b_16 --fp8 --steps 5 --warmup 3
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r46_autotune_gfx950.json
run r46_bench_a.txt 400 python bench.py
run r46_bench_b.txt 400 python bench.py
run r46_bench_256.txt 400 python bench.py --batch 256
run r46_bench_vit8.txt 400 python bench.py --model vit_b_16 --fp8 --steps 10 --warmup 5
exit 0
