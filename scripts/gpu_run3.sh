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
run r3_tests.txt 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r3_bench_native.txt 300 python bench.py --backend native --steps 20 --warmup 5
run r3_bench_native_graph.txt 300 python bench.py --backend native --steps 20 --warmup 5 --graph
run r3_bench_torch_graph.txt 300 python bench.py --backend torch --steps 20 --warmup 5 --graph
export TMPDIR=/tmp
run r3_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native -o run --output-format csv -- python3 bench.py --backend native --steps 5 --warmup 3
run r3_kbench.txt 300 python scripts/bench_kernels.py --iters 5
exit 0
