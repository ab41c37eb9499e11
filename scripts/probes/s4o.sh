source scripts/gpurun_lib.sh
bash scripts/trainer_graph_ab.sh s4o 256 60 && \
run s4o_bench.txt 400 python bench.py && \
run s4o_bench_eager.txt 400 python bench.py --eager && \
run s4o_bench512.txt 400 python bench.py --batch 512 && \
run s4o_bench512_eager.txt 400 python bench.py --batch 512 --eager
