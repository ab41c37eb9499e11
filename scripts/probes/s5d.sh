source scripts/gpurun_lib.sh
PDT_TUNE_ROUNDS=6 PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=$PWD/gpurun_out/tune_r50c.json run s5d_retune.txt 900 python bench.py --steps 5 --warmup 3 && \
cp gpurun_out/tune_r50c.json /tmp/tune_c.json && \
run s5d_shipped_1.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_c.json PDT_AUTOTUNE=0 run s5d_fresh_1.txt 400 python bench.py && \
run s5d_shipped_2.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_c.json PDT_AUTOTUNE=0 run s5d_fresh_2.txt 400 python bench.py
