#!/bin/bash
# Round 4: 1024-thread partial-amax roll (LayerNorm fp8 outputs) -- fp8 tests, ViT A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4tt
run ${T}_tests.txt 400 python -u -m pytest tests/test_vit_fusion_gpu.py tests/test_kernels_gpu.py tests/test_attention_bwd_f8_gpu.py -k "vit or ln or fp8 or f8 or attention" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
for i in 1 2; do
PDT_ROLL_NT=256 run ${T}_vit_off$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_on$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
