source scripts/gpurun_lib.sh
run r50_bench_tune.txt 600 python bench.py --steps 10 --warmup 5
run r50_bench_tune256.txt 600 python bench.py --steps 10 --warmup 5 --batch 256
run r50_bench_tunevit.txt 600 python bench.py --model vit_b_16 --fp8 --steps 5 --warmup 3
run r50_bench_tunevit16.txt 600 python bench.py --model vit_b_16 --steps 5 --warmup 3
run r50_bench_tune152.txt 600 python bench.py --model resnet152 --batch 512 --steps 5 --warmup 3
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r50_autotune_gfx950.json
run r50_bench_a.txt 400 python bench.py
run r50_bench_b.txt 400 python bench.py
run r50_bench_256.txt 400 python bench.py --batch 256
run r50_bench_vit8.txt 400 python bench.py --model vit_b_16 --fp8 --steps 10 --warmup 5
exit 0
