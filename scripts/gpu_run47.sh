source scripts/gpurun_lib.sh
run r47_probe.txt 300 python scripts/probe_linear_wgrad.py
exit 0
