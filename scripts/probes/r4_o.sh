#!/bin/bash
# Round 4: fp8 weight-gradient bias sums spread over the split's tile columns -- tests, ViT A/B
# (old plan vs new plan + spread bias), kernel trace.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4o
run ${T}_tests.txt 300 python -u -m pytest tests/test_vit_fusion_gpu.py -k "wgrad or mlp or vit" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
for i in 1 2; do
PDT_WG8_PLAN=0 run ${T}_vit_old$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_new$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
