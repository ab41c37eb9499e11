set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))" > gpurun_out/devinfo.txt 2>&1
MODE=autocast timeout -k 10 300 python scripts/probe_stock.py > gpurun_out/probe_autocast.txt 2>&1
MODE=bf16 timeout -k 10 300 python scripts/probe_stock.py > gpurun_out/probe_bf16.txt 2>&1
cd /tmp && export TMPDIR=/tmp
MODE=autocast STEPS=5 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_stock -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/probe_stock.py > $GRAFT_REPO_ROOT/gpurun_out/prof_stock.log 2>&1
