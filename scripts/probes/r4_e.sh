#!/bin/bash
# Round 4: persistent ring tiles (conv_nt ids 45-46), the halo stem, the AX fold on tiles 30/31: correctness, per-variant GEMM times,
# targeted re-tune of the ResNet-50 bs2048 table against them, bench with the re-tuned table.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4e
run ${T}_tests_pers.txt 400 python -u -m pytest tests/test_conv_persistent_gpu.py tests/test_stem_gpu.py tests/test_bn_fold_gpu.py -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${T}_tests_pers.txt && ! grep -q "failed" gpurun_out/${T}_tests_pers.txt || { echo "persistent tests failed"; exit 1; }
run ${T}_bench_gemm.txt 300 python scripts/bench_gemm.py --shapes resnet --variants 34,35,36,37,45,46 || exit $?
run ${T}_bench_gemm_vit.txt 300 python scripts/bench_gemm.py --variants 34,35,36,37,45,46 || exit $?
PDT_RETUNE_AX=30,31 bash scripts/gpu_job.sh $T retunewith:r50pers:45-46 || exit $?
PDT_AUTOTUNE_CACHE=$PWD/gpurun_out/tune_r50pers.json run ${T}_bench_pers.txt 400 python bench.py || exit $?
run ${T}_bench_base.txt 400 python bench.py || exit $?
