source scripts/gpurun_lib.sh
run r58_stem.txt 300 python -u -m pytest tests/test_bn_fusion_gpu.py -k stem -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider
run r58_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_58 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
run r58_bench_a.txt 400 python bench.py
PDT_STEM_POOL_BWD_FUSED=0 run r58_bench_unf.txt 400 python bench.py
run r58_bench_b.txt 400 python bench.py
PDT_STEM_POOL_BWD_FUSED=0 run r58_bench_unf_b.txt 400 python bench.py
run r58_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run r58_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
