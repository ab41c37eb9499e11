source scripts/gpurun_lib.sh
run r33_vtimes.txt 600 python scripts/variant_times.py
exit 0
