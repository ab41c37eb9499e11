source scripts/gpurun_lib.sh
run r23_bench_r50_A.txt 300 python bench.py --steps 30 --warmup 10
PDT_AUTOTUNE_CACHE=/tmp/t33.json PDT_NT_VARIANTS=0-33 run r23_bench_r50_B.txt 400 python bench.py --steps 30 --warmup 10
PDT_AUTOTUNE_CACHE=/tmp/t29.json PDT_NT_VARIANTS=0-29 run r23_bench_r50_C.txt 400 python bench.py --steps 30 --warmup 10
run r23_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_23 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
PDT_AUTOTUNE_CACHE=/tmp/t29.json PDT_NT_VARIANTS=0-29 run r23_prof_r50C.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_23C -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
cp /tmp/t33.json gpurun_out/autotune_t33.json; cp /tmp/t29.json gpurun_out/autotune_t29.json
run r23_tests.txt 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider -k "fp8 or f8 or vit"
run r23_bench_vit8.txt 500 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
exit 0
