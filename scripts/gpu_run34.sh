source scripts/gpurun_lib.sh
run r34_tests.txt 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run r34_bench_r50a.txt 400 python bench.py --steps 30 --warmup 10
run r34_bench_r50b.txt 300 python bench.py --steps 30 --warmup 10
run r34_bench_vit8.txt 500 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
run r34_bench_r152.txt 500 python bench.py --model resnet152 --batch 512 --steps 10 --warmup 5
run r34_prof_r50.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_34 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3
exit 0
