source scripts/gpurun_lib.sh
run s4g_fold_tests.txt 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "bn_fold or bn_fusion or bottleneck" && \
run s4g_op.txt 600 python -u scripts/op_profile.py --top 60 && \
run s4g_op_off.txt 600 python -u scripts/op_profile.py --top 60 --set PDT_FUSE_BN_BWD2=0 && \
run s4g_bench.txt 400 python bench.py
