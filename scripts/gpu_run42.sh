source scripts/gpurun_lib.sh
run r42_bench_b512.txt 500 python bench.py --steps 20 --warmup 8 --batch 512
run r42_bench_b384.txt 500 python bench.py --steps 20 --warmup 8 --batch 384
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r42_autotune_gfx950.json
run r42_bench_b512_torch.txt 600 python bench.py --steps 20 --warmup 8 --batch 512 --backend torch
run r42_bench_b256_torch.txt 600 python bench.py --steps 20 --warmup 8 --batch 256 --backend torch
exit 0
