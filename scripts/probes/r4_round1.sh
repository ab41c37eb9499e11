#!/bin/bash
# Round-4 first GPU session: GEMM lab timings + counters, bench (native reducer) and its
# torch-DDP A/B, a kernel trace of the bench step, the GPU test suite, smoke.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4b
bash scripts/gemm_lab/run.sh $T pmc 1 || exit $?
run ${T}_bench_native.txt 400 python bench.py || exit $?
PDT_DDP=torch run ${T}_bench_torchddp.txt 400 python bench.py || exit $?
bash scripts/gpu_job.sh $T ktrace tests smoke
