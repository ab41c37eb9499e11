source scripts/gpurun_lib.sh
run r14_f8.txt 300 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k "fp8 or f8"
run r14_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r14_bench_r50.txt 300 python bench.py --steps 30 --warmup 10
PDT_AUTOTUNE_CACHE=/tmp/t29.json PDT_NT_VARIANTS=0-29 run r14_bench_r50_v29.txt 400 python bench.py --steps 30 --warmup 10
PDT_AUTOTUNE_CACHE=/tmp/tall.json run r14_bench_r50_vall.txt 400 python bench.py --steps 30 --warmup 10
run r14_bench_vit.txt 400 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r14_bench_vit_fp8.txt 400 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
cp /tmp/t29.json gpurun_out/autotune_v29.json; cp /tmp/tall.json gpurun_out/autotune_vall.json
exit 0
