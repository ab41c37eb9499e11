source scripts/gpurun_lib.sh
run s4i_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "bn_fold or stem or s2d" && \
run s4i_op.txt 600 python -u scripts/op_profile.py --top 70 && \
run s4i_bench.txt 400 python bench.py && \
run s4i_bench_eager.txt 400 python bench.py --eager
