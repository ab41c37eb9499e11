source scripts/gpurun_lib.sh
run r10_kbench_plain.txt 400 python scripts/bench_kernels.py --iters 5
PDT_NT_STORE=1 run r10_kbench_nt.txt 400 python scripts/bench_kernels.py --iters 5
run r10_bench_r50.txt 300 python bench.py --steps 30 --warmup 10
PDT_NT_STORE=1 run r10_bench_r50_nt.txt 300 python bench.py --steps 30 --warmup 10
run r10_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native10 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
exit 0
