source scripts/gpurun_lib.sh
run r55_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run r55_bench_a.txt 400 python bench.py
run r55_bench_b.txt 400 python bench.py
run r55_bench_256.txt 400 python bench.py --batch 256
run r55_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_55 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
