source scripts/gpurun_lib.sh
run r43_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()"
run r43_bench_a.txt 400 python bench.py
run r43_bench_b.txt 400 python bench.py --steps 30 --warmup 10
run r43_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_43 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
