#!/bin/bash
# Round 4: MLP fc2 data gradient on the library GEMM + one gelu'-multiply / e5m2 cast / bias-sum
# pass, vs the native tile with that epilogue -- tests, ViT A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4rr
run ${T}_tests.txt 400 python -u -m pytest tests/test_vit_fusion_gpu.py tests/test_kernels_gpu.py -k "vit or mlp or gelu or f8" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
for i in 1 2; do
PDT_FC2_DGRAD_LIB=0 run ${T}_vit_off$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_on$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
