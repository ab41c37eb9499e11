#!/bin/bash
# Round 4: persistent fp8 attention backward (next head prefetched across the dQ phase) -- tests, ViT fp8 A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4k
run ${T}_tests.txt 400 python -u -m pytest tests/test_attention_bwd_f8_gpu.py tests/test_vit_fusion_gpu.py -k "attention" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
PDT_ATTN_BWD_PERSIST=0 run ${T}_vit_base.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_pers.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
PDT_ATTN_BWD_PERSIST=0 run ${T}_vit_base2.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_pers2.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
