source scripts/gpurun_lib.sh
run r29_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()"
run r29_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run r29_bench_r50a.txt 300 python bench.py --steps 30 --warmup 10
run r29_bench_r50_torch.txt 300 python bench.py --steps 20 --warmup 10 --backend torch
run r29_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_29 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
