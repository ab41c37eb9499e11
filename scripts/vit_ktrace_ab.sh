set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in 1 0; do
  d=gpurun_out/s3t_kt_bwd$mode
  PDT_FP8_ATTN_BWD=$mode timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --model vit_b_16 --fp8 --steps 3 --warmup 3 > gpurun_out/s3t_kt_bwd$mode.log 2>&1
  f=$(find $d -name '*kernel_trace.csv' | head -n 1)
  python scripts/step_profile.py "$f" --top 25 > gpurun_out/s3t_kt_bwd${mode}_step.txt 2>&1
  rm -rf $d
done
