source scripts/gpurun_lib.sh
run s4k_vit_graph.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 && \
run s4k_vit_eager.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 --eager && \
run s4k_vit_graph2.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5
