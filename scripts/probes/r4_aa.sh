#!/bin/bash
# Round 4: qkv bias gradient from the e5m2 cast of its output gradient -- tests, ViT A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4aa
run ${T}_tests.txt 400 python -u -m pytest tests/test_vit_fusion_gpu.py tests/test_kernels_gpu.py -k "vit or mlp or fp8 or f8 or ln" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
for i in 1 2; do
PDT_CAST_DB=0 run ${T}_vit_off$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_on$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
