#!/bin/bash
# Round 4: per-call roofline gap table of the ResNet-50 bs2048 step, GEMM side-by-side
# (native vs hipBLASLt / _scaled_mm on the ViT shapes), lab on the ResNet GEMM shapes.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4c
run ${T}_opprof.txt 400 python scripts/op_profile.py --batch 2048 --steps 2 --warmup 3 --top 80 --gap 60 || exit $?
run ${T}_bench_gemm.txt 300 python scripts/bench_gemm.py || exit $?
B=scripts/gemm_lab/gemm_lab
run ${T}_lab_r50.txt 200 bash -c "$B 401408 256 1024 10 1 4 7 8 10 && $B 401408 1024 256 10 1 4 7 8 10 && $B 100352 512 2048 10 1 4 7 8 && $B 100352 2048 512 10 1 4 7 8 && $B 6422528 64 256 5 10 11 12 && $B 6422528 256 64 5 1 4 7" || exit $?
