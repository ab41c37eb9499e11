source scripts/gpurun_lib.sh
run s4y_dbg.txt 900 python -u scripts/probes/graph_ddp_debug.py && \
run s4y_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "hip_graph"
