source scripts/gpurun_lib.sh
run r61_bench_256.txt 400 python bench.py --batch 256
PDT_STEM_S2D=0 run r61_bench_256_direct.txt 400 python bench.py --batch 256
run r61_bench_256_b.txt 400 python bench.py --batch 256
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r61_autotune.json
run r61_prof256.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_61 -o run --output-format csv -- python3 bench.py --batch 256 --steps 5 --warmup 3
PDT_STEM_S2D=0 run r61_prof256d.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_61d -o run --output-format csv -- python3 bench.py --batch 256 --steps 5 --warmup 3
exit 0
