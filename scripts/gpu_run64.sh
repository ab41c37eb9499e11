source scripts/gpurun_lib.sh
run r64_pytest_gpu.txt 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run r64_bench.txt 400 python bench.py
run r64_bench_b.txt 400 python bench.py
run r64_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r64 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
