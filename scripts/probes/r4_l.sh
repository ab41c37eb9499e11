#!/bin/bash
# Round 4: MLP fc1 on the library GEMM + one GELU-dual/fp8-cast pass vs the fused native epilogue.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4l
run ${T}_tests.txt 400 python -u -m pytest tests/test_vit_fusion_gpu.py tests/test_kernels_gpu.py -k "mlp or gelu or vit" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
for i in 1 2; do
PDT_FP8_FC1_LIB=0 run ${T}_vit_fused$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
PDT_FP8_FC1_LIB=1 run ${T}_vit_lib$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
PDT_FP8_FC1_LIB=1 bash scripts/gpu_job.sh $T ktrace:--model,vit_b_16,--fp8,--batch,1024
