#!/bin/bash
# Round 4: hardware counters of the fp8 weight-gradient tiles (v12 register-staged 8-wave 256x256,
# v20 its LDS-DMA ring, v24 the 4-wave LDS-DMA ring) on the ViT bs1024 shapes.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4m
LIST=gpurun_out/${T}_counters.txt
timeout -k 10 120 rocprofv3 -L > $LIST 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
have() { grep -qw "$1" $LIST; }
pick() { local out=""; for c in "$@"; do have $c && out="$out $c"; done; echo $out; }
P1=$(pick SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE)
P2=$(pick SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum)
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  echo "pass $i: $P"
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${T}_pmc$i -o run -- \
    python3 scripts/bench_f8.py --fwd "" --wgrad 12,20,24 --iters 3 > gpurun_out/${T}_pmc$i.log 2>&1
  rc=$?
  echo "[pass $i rc=$rc] $P" | tee -a gpurun_out/${T}_pmc$i.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
