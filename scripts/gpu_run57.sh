source scripts/gpurun_lib.sh
run r57_stem.txt 300 python -u -m pytest tests/test_bn_fusion_gpu.py -k stem -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider
run r57_prof_s2d.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_57s -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
PDT_STEM_S2D=0 run r57_prof_direct.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_57d -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
run r57_bench_s2d.txt 400 python bench.py
PDT_STEM_S2D=0 run r57_bench_direct.txt 400 python bench.py
run r57_bench_s2d_b.txt 400 python bench.py
PDT_STEM_S2D=0 run r57_bench_direct_b.txt 400 python bench.py
run r57_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
exit 0
