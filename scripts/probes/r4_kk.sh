#!/bin/bash
# Round 4: from-scratch tuning pass of every ResNet-50 bs2048 key on the final kernels, then the
# shipped table vs the fresh one on the same box.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4kk
PDT_TUNE_ROUNDS=3 PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=gpurun_out/tune_r50_r4kk.json run ${T}_tune.txt 1000 python bench.py --steps 3 --warmup 2 || exit $?
for i in 1 2; do
run ${T}_r50_shipped$i.txt 400 python bench.py || exit $?
PDT_AUTOTUNE=0 PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=gpurun_out/tune_r50_r4kk.json run ${T}_r50_fresh$i.txt 400 python bench.py || exit $?
done
