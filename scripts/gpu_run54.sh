source scripts/gpurun_lib.sh
run r54_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -s
run r54_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_54 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
