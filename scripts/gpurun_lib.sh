# Shared helper for GPU scripts: each GPU step under its own timeout; stop the
# whole call on a crash / timeout / GPU fault message in the step's log.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <logfile> <timeout> cmd...
  local log=$1; local t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[rc=$rc] $*" >> gpurun_out/$log
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $log"; exit $rc; fi
  if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" gpurun_out/$log; then
    echo "GPU fault reported in $log -- stopping"; exit 99
  fi
  return 0
}
