#!/bin/bash
# Round 4: the ViT blocks' residual adds in the next LayerNorm kernel (proj / fc2 as plain GEMMs
# on the library path) -- tests, ViT fp8 bs1024 A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4s
run ${T}_tests.txt 400 python -u -m pytest tests/test_vit_fusion_gpu.py tests/test_kernels_gpu.py -k "vit or ln or mlp or fp8" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
for i in 1 2; do
PDT_LN_ADD=0 run ${T}_vit_epi$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_ln$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
