source scripts/gpurun_lib.sh
run s4l_tests.txt 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "halo" && \
run s4l_halo.txt 600 python -u scripts/halo_times.py 2048
