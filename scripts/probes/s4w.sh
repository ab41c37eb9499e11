source scripts/gpurun_lib.sh
run s4w_tests.txt 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "hip_graph or graph_collectives or rccl"
