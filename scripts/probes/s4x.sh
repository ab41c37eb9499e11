source scripts/gpurun_lib.sh
run s4x_dbg.txt 1100 python -u scripts/probes/graph_ddp_debug.py
