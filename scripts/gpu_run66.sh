source scripts/gpurun_lib.sh
run r66_bench_gloo2.txt 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 3 --batch 64 --dist-backend gloo
run r66_bench_r152.txt 400 python bench.py --model resnet152 --steps 15 --warmup 5
run r66_bench_vit.txt 400 python bench.py --model vit_b_16 --steps 20 --warmup 5
run r66_bench_vit_fp8.txt 400 python bench.py --model vit_b_16 --fp8 --steps 20 --warmup 5
exit 0
