source scripts/gpurun_lib.sh
cp profiles/tune_r50_round3_s4s.json /tmp/tune_fresh.json
run s4t_shipped_1.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_fresh.json PDT_AUTOTUNE=0 run s4t_fresh_1.txt 400 python bench.py && \
run s4t_shipped_2.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_fresh.json PDT_AUTOTUNE=0 run s4t_fresh_2.txt 400 python bench.py
