#!/bin/bash
# Round 4: unclamped in-range e4m3 conversions in the fp8 attention kernels -- tests, ViT bench, trace.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4u
run ${T}_tests.txt 400 python -u -m pytest tests/test_attention_bwd_f8_gpu.py tests/test_vit_fusion_gpu.py -k "attention or vit" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
run ${T}_vit1.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit2.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
