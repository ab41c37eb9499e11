#!/bin/bash
# Round 4: persistent fp8 attention backward (next head prefetched across the dQ phase) and the
# dual-GELU MLP epilogues (act 4 / 5) -- tests, then ViT fp8 bs1024 A/B/C on one box.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4k
run ${T}_tests.txt 500 python -u -m pytest tests/test_attention_bwd_f8_gpu.py tests/test_vit_fusion_gpu.py tests/test_kernels_gpu.py -k "attention or gelu or mlp or vit or f8" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
for i in 1 2; do
PDT_ATTN_BWD_PERSIST=0 PDT_GELU_DUAL=0 run ${T}_vit_base$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
PDT_GELU_DUAL=0 run ${T}_vit_pers$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_both$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
