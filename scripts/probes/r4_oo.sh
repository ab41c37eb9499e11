#!/bin/bash
# Round 4: library fc1 keeps its pre-activation output (gelu' formed in the fc2 data-gradient
# epilogue, act 3) instead of the cast pass writing gelu'(z) -- tests, tune, ViT A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4oo
run ${T}_tests.txt 400 python -u -m pytest tests/test_vit_fusion_gpu.py tests/test_kernels_gpu.py -k "vit or mlp or gelu or f8" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
export PDT_AUTOTUNE_CACHE=gpurun_out/tune_fc1pre_r4oo.json
run ${T}_vit_tune.txt 600 python bench.py --model vit_b_16 --fp8 --steps 3 --warmup 2 || exit $?
for i in 1 2; do
PDT_FC1_KEEP_PRE=0 run ${T}_vit_off$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_on$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
