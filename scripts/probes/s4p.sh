source scripts/gpurun_lib.sh
run s4p_vit_graph.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 --graph && \
run s4p_vit_eager.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 --eager && \
run s4p_vit_graph2.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 --graph
