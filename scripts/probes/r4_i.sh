#!/bin/bash
# Round 4: 4-wave stem weight gradient back; fused pool-backward + BN reduction A/B (same box).
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4i
run ${T}_tests.txt 300 python -u -m pytest tests/test_stem_gpu.py -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
PDT_POOL_BNRED=0 run ${T}_bench_sep.txt 400 python bench.py || exit $?
run ${T}_bench_fused.txt 400 python bench.py || exit $?
PDT_POOL_BNRED_BLOCKS=2048 run ${T}_bench_fused2048.txt 400 python bench.py || exit $?
PDT_POOL_BNRED=0 run ${T}_bench_sep2.txt 400 python bench.py || exit $?
run ${T}_bench_fused2.txt 400 python bench.py || exit $?
bash scripts/gpu_job.sh $T ktrace bench:--model,vit_b_16,--fp8 ktrace:--model,vit_b_16,--fp8,--batch,1024
