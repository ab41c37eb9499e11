#!/bin/bash
# Hardware-counter passes over a short bench.py run, one rocprofv3 --pmc run per
# pass (counter slots per pass on gfx950: 8 SQ, 4 TCC with FETCH_SIZE = 3 and
# WRITE_SIZE = 2, 2 GRBM). Requested counters the agent does not offer
# (`rocprofv3 -L`) are dropped so a renamed counter cannot fail the call.
#
#   gpurun -- bash scripts/pmc_passes.sh TAG [bench.py args...]
#
# Output: gpurun_out/TAG_pmc<i>/run_counter_collection.csv per pass; summarise
# with scripts/pmc_summary.py.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
LIST=gpurun_out/${TAG}_counters.txt
timeout -k 10 120 rocprofv3 -L > $LIST 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
have() { grep -qw "$1" $LIST; }
pick() { local out=""; for c in "$@"; do have $c && out="$out $c"; done; echo $out; }
P1=$(pick SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE)
P2=$(pick SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum)
P3=$(pick FETCH_SIZE)
P4=$(pick WRITE_SIZE)
echo "pass1: $P1"; echo "pass2: $P2"; echo "pass3: $P3"; echo "pass4: $P4"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i + 1))
  [ -z "$P" ] && continue
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_pmc$i -o run -- \
    python3 bench.py --steps 2 --warmup 2 "$@" > gpurun_out/${TAG}_pmc$i.log 2>&1
  rc=$?
  echo "[pass $i rc=$rc] $P" | tee -a gpurun_out/${TAG}_pmc$i.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
