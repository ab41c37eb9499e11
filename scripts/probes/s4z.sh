source scripts/gpurun_lib.sh
run s4z_g1.txt 400 python bench.py && \
run s4z_e1.txt 400 python bench.py --eager && \
run s4z_g2.txt 400 python bench.py && \
run s4z_g512.txt 400 python bench.py --batch 512
