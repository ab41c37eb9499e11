#!/bin/bash
# Round 4: wave-aware split planning of the fp8 weight gradient -- tests, per-shape times (old /
# new plan), ViT fp8 bs1024 A/B.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4n
run ${T}_tests.txt 300 python -u -m pytest tests/test_vit_fusion_gpu.py -k "wgrad or mlp" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
PDT_WG8_PLAN=0 run ${T}_f8_old.txt 300 python scripts/bench_f8.py --fwd "" --wgrad 10,12,19,20 || exit $?
run ${T}_f8_new.txt 300 python scripts/bench_f8.py --fwd "" --wgrad 10,12,19,20 || exit $?
for i in 1 2; do
PDT_WG8_PLAN=0 run ${T}_vit_old$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
run ${T}_vit_new$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
for i in 1 2; do
PDT_WG_PLAN=0 run ${T}_r50_old$i.txt 400 python bench.py || exit $?
run ${T}_r50_new$i.txt 400 python bench.py || exit $?
done
