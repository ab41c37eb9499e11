#!/bin/bash
# GPU side of the GEMM lab: timing over a few shapes, then optional counter passes.
#   gpurun -- bash scripts/gemm_lab/run.sh TAG [pmc]
source "$(dirname "$0")/../gpurun_lib.sh"
TAG=$1; shift
B=scripts/gemm_lab/gemm_lab
run ${TAG}_lab_8k.txt 120 $B 8192 8192 8192 10
run ${TAG}_lab_4k.txt 120 $B 4096 4096 4096 20
run ${TAG}_lab_r50s3.txt 120 $B 401408 256 1024 10
run ${TAG}_lab_r50s3b.txt 120 $B 401408 1024 256 10
run ${TAG}_lab_vit.txt 120 $B 50432 3072 768 10
if [ "$1" == "pmc" ]; then
  shift
  V=${1:-0}
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    run ${TAG}_lab_pmc$i.txt 90 timeout -s KILL 80 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_lab_pmc$i -o run -- $B 8192 8192 8192 3 $V
  done
fi
