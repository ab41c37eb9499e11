source scripts/gpurun_lib.sh
run s5c_r152.txt 600 python bench.py --model resnet152 --batch 2048 --steps 5 --warmup 3 && \
run s5c_vit.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5
