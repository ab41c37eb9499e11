#!/bin/bash
# Round 4: ViT patch embedding as patchify + K=768 GEMM (vs the channel-padded K=2048 implicit
# GEMM) -- tests, tune the new keys, ViT A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4ll
run ${T}_tests.txt 400 python -u -m pytest tests/test_vit_fusion_gpu.py tests/test_fallback_gpu.py -k "patch or vit" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
export PDT_AUTOTUNE_CACHE=gpurun_out/tune_patch_r4ll.json
run ${T}_vit_tune.txt 600 python bench.py --model vit_b_16 --fp8 --steps 3 --warmup 2 || exit $?
for i in 1 2; do
PDT_PATCH_LINEAR=0 run ${T}_vit_off$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_on$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
