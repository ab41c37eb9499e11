source scripts/gpurun_lib.sh
run r52_bench_x1.txt 400 python bench.py
PDT_WGRAD_XCD=0 run r52_bench_x0.txt 400 python bench.py
run r52_bench_x1b.txt 400 python bench.py
PDT_WGRAD_XCD=0 run r52_bench_x0b.txt 400 python bench.py
run r52_vit_x1.txt 400 python bench.py --model vit_b_16 --fp8 --steps 10 --warmup 5
PDT_WGRAD_XCD=0 run r52_vit_x0.txt 400 python bench.py --model vit_b_16 --fp8 --steps 10 --warmup 5
exit 0
