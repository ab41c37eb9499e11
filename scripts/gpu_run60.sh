source scripts/gpurun_lib.sh
run r60_stem.txt 300 python -u -m pytest tests/test_bn_fusion_gpu.py -k stem -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run r60_bench_r50.txt 400 python bench.py
run r60_bench_r50_256.txt 400 python bench.py --batch 256
run r60_bench_r152.txt 500 python bench.py --model resnet152 --batch 512 --steps 15 --warmup 5
run r60_bench_vit.txt 500 python bench.py --model vit_b_16 --steps 20 --warmup 5
run r60_bench_vit_fp8.txt 500 python bench.py --model vit_b_16 --fp8 --steps 20 --warmup 5
run r60_bench_r50_b.txt 400 python bench.py
exit 0
