source scripts/gpurun_lib.sh
run r59_stem.txt 300 python -u -m pytest tests/test_bn_fusion_gpu.py tests/test_kernels_gpu.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider
run r59_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_59 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
PDT_POOL_BN_BLOCKS=16384 run r59_prof16k.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_59b -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
run r59_bench_a.txt 400 python bench.py
PDT_STEM_POOL_BWD_FUSED=0 run r59_bench_unf.txt 400 python bench.py
run r59_bench_b.txt 400 python bench.py
PDT_STEM_POOL_BWD_FUSED=0 run r59_bench_unf_b.txt 400 python bench.py
exit 0
