source scripts/gpurun_lib.sh
run r56_stem.txt 300 python -u -m pytest tests/test_bn_fusion_gpu.py tests/test_train_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run r56_bench_s2d.txt 400 python bench.py
PDT_STEM_S2D=0 run r56_bench_direct.txt 400 python bench.py
run r56_bench_s2d_b.txt 400 python bench.py
run r56_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
exit 0
