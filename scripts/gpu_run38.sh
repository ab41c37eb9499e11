source scripts/gpurun_lib.sh
run r38_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run r38_bench_a.txt 400 python bench.py --steps 30 --warmup 10
run r38_bench_b.txt 300 python bench.py --steps 30 --warmup 10
PDT_FUSE_BN_BWD=0 run r38_bench_nofuse.txt 300 python bench.py --steps 30 --warmup 10
run r38_bench_r152.txt 500 python bench.py --model resnet152 --batch 512 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/r38_autotune_gfx950.json
run r38_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_38 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
