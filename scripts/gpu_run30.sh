source scripts/gpurun_lib.sh
run r30_tests.txt 600 python -u -m pytest tests/test_train_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run r30_bench_gloo2.txt 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 3 --batch 64 --dist-backend gloo
run r30_kbench.txt 900 python scripts/bench_kernels.py --iters 5
run r30_bench_r50_torch.txt 600 python bench.py --steps 20 --warmup 10 --backend torch
exit 0
