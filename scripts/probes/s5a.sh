source scripts/gpurun_lib.sh
cp profiles/tune_shipped_before_retune_round3.json /tmp/tune_old.json
run s5a_new_1.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_old.json PDT_AUTOTUNE=0 run s5a_old_1.txt 400 python bench.py && \
run s5a_new_2.txt 400 python bench.py && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_old.json PDT_AUTOTUNE=0 run s5a_old_2.txt 400 python bench.py
