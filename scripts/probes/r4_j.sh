#!/bin/bash
# Round 4: fp8 library path (hipBLASLt) for the plain ViT GEMMs -- tests, then ViT fp8 bs1024 A/B on one box.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4j
run ${T}_tests.txt 300 python -u -m pytest tests/test_kernels_gpu.py -k "f8 or fp8" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
PDT_FP8_LIB=0 run ${T}_vit_native.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_lib.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
PDT_FP8_LIB=0 run ${T}_vit_native2.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_lib2.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
