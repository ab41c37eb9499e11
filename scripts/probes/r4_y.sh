#!/bin/bash
# Round 4: wave-aware split plan for the one-workgroup-per-CU bf16 weight-gradient tiles, and a
# targeted re-tune of the ResNet-50 bs2048 wgrad keys against those tiles; A/B on one box.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4y
run ${T}_tests.txt 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/tune_wg_r4y.json
PDT_RETUNE_WG=12-17,23-27 PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=gpurun_out/tune_wg_r4y.json run ${T}_retune.txt 900 python bench.py --steps 3 --warmup 2 || exit $?
for i in 1 2; do
run ${T}_r50_shipped$i.txt 400 python bench.py || exit $?
PDT_AUTOTUNE=0 PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=gpurun_out/tune_wg_r4y.json run ${T}_r50_retuned$i.txt 400 python bench.py || exit $?
done
