#!/bin/bash
# Round 4 / BASELINE config 4: ResNet-152 native at the HBM-sized batch (2560: the stem's
# N x 112 x 112 x 64 activation stays under the 2^31-element kernel index limit) and at 2048,
# and the stock stack at 2048 with the MIOpen find db seeded from the ResNet-50 bs-2048 one
# (ResNet-152's bottleneck conv shapes are ResNet-50's).
source "$(dirname "$0")/../gpurun_lib.sh"
T=${1:-r4r}
run ${T}_r152_native_2560.txt 400 python bench.py --model resnet152 --batch 2560 --steps 10 --warmup 5 || exit $?
run ${T}_r152_native_2048.txt 400 python bench.py --model resnet152 --batch 2048 --steps 10 --warmup 5 || exit $?
bash scripts/gpu_job.sh $T benchlong:--model,resnet152,--backend,torch,--batch,2048,--steps,10,--warmup,5
