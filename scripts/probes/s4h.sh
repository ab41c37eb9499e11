source scripts/gpurun_lib.sh
run s4h_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "bn_fold or hip_graph or bottleneck" && \
run s4h_op.txt 600 python -u scripts/op_profile.py --top 60 && \
run s4h_op_off.txt 600 python -u scripts/op_profile.py --top 60 --set PDT_FUSE_BN_BWD2=0 && \
run s4h_bench.txt 400 python bench.py && \
run s4h_bench_vit.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5
