#!/bin/bash
# Round 4: halo stem forward + weight gradient: tests; A/B on one
# box (bench with the merged table, PDT_STEM_HALO=0 vs default); kernel trace of the step.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4g
run ${T}_tests_pers.txt 300 python -u -m pytest tests/test_stem_gpu.py -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests_pers.txt && ! grep -q "failed" gpurun_out/${T}_tests_pers.txt || { echo "tests failed"; exit 1; }
PDT_STEM_HALO=0 run ${T}_bench_nohalo.txt 400 python bench.py || exit $?
run ${T}_bench_halo.txt 400 python bench.py || exit $?
PDT_STEM_HALO=0 run ${T}_bench_nohalo2.txt 400 python bench.py || exit $?
run ${T}_bench_halo2.txt 400 python bench.py || exit $?
bash scripts/gpu_job.sh $T ktrace
