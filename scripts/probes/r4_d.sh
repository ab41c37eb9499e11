#!/bin/bash
# Round 4: two-workgroups-per-CU GEMM (lab v8) vs the 256x256 ring on the ResNet / ViT GEMM shapes;
# production native vs hipBLASLt on the same ResNet shapes.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4d
B=scripts/gemm_lab/gemm_lab
run ${T}_lab.txt 300 bash -c "$B 401408 256 1024 10 4 7 13 14 15 16 && $B 401408 1024 256 10 4 7 13 14 15 16 && $B 100352 512 2048 10 4 7 13 14 15 16 && $B 100352 2048 512 10 4 7 13 14 15 16 && $B 1605632 512 128 10 4 7 13 14 15 16 && $B 50432 3072 768 10 4 7 13 14 15 16 && $B 50432 768 3072 10 13 14 15 16 && $B 8192 8192 8192 5 4 13 14 16" || exit $?
run ${T}_bench_gemm_resnet.txt 300 python scripts/bench_gemm.py --shapes resnet || exit $?
