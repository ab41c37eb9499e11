source scripts/gpurun_lib.sh
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=$PWD/gpurun_out/tune_r50b.json run s4u_retune.txt 600 python bench.py --steps 5 --warmup 3 --eager && \
cp gpurun_out/tune_r50b.json /tmp/tune_b.json && \
run s4u_shipped_1.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_b.json PDT_AUTOTUNE=0 run s4u_fresh_1.txt 400 python bench.py && \
run s4u_shipped_2.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_b.json PDT_AUTOTUNE=0 run s4u_fresh_2.txt 400 python bench.py
