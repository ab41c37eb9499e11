source scripts/gpurun_lib.sh
run s4q_eager.txt 400 python bench.py --eager && \
HIP_FORCE_DEV_KERNARG=1 run s4q_eager_devka.txt 400 python bench.py --eager && \
run s4q_graph.txt 400 python bench.py && \
HIP_FORCE_DEV_KERNARG=1 run s4q_graph_devka.txt 400 python bench.py
