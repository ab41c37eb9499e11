#!/bin/bash
# Round 4: 8-wave stem weight gradient (tests, trace), gradient readiness at the bench batch.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4h
run ${T}_tests.txt 300 python -u -m pytest tests/test_stem_gpu.py -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests.txt && ! grep -q "failed" gpurun_out/${T}_tests.txt || { echo "tests failed"; exit 1; }
bash scripts/gpu_job.sh $T ktrace bench py:scripts/grad_ready_order.py:--batch,2048 || exit $?
