#!/bin/bash
# Round 4: validation (whole GPU suite, smoke, ResNet-50 bench) + a from-scratch tuning pass of the
# ViT-B/16 fp8 bs1024 keys (the library ids and the wave-aware wgrad plan included), then the ViT
# bench with the shipped table vs the fresh one on the same box.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4r
bash scripts/gpu_job.sh $T tests smoke bench || exit $?
export PDT_FP8_FC1_LIB=1
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=gpurun_out/tune_vit_r4r.json run ${T}_vit_tune.txt 600 python bench.py --model vit_b_16 --fp8 --steps 5 --warmup 3 || exit $?
for i in 1 2; do
run ${T}_vit_shipped$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
PDT_AUTOTUNE=0 PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=gpurun_out/tune_vit_r4r.json run ${T}_vit_fresh$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
