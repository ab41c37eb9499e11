# Each GPU step under its own timeout; stop the whole call on a crash/timeout.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # run <logfile> <timeout> cmd...
  local log=$1; local t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$log 2>&1
  local rc=$?
  echo "[rc=$rc] $*" >> gpurun_out/$log
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $log"; exit $rc; fi
  return 0
}
run r2_tests.txt 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider
run r2_kbench.txt 300 python scripts/bench_kernels.py --iters 5
run r2_bench_native.txt 300 python bench.py --backend native --steps 20 --warmup 5
run r2_bench_torch.txt 300 python bench.py --backend torch --steps 20 --warmup 5
exit 0
