source scripts/gpurun_lib.sh
run r39_kbench.txt 600 python scripts/bench_kernels.py --iters 5
exit 0
