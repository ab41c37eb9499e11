source scripts/gpurun_lib.sh
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=$PWD/gpurun_out/tune_vit.json run s4v_retune.txt 900 python bench.py --model vit_b_16 --fp8 --steps 5 --warmup 3 && \
cp gpurun_out/tune_vit.json /tmp/tune_v.json && \
run s4v_shipped_1.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_v.json PDT_AUTOTUNE=0 run s4v_fresh_1.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 && \
run s4v_shipped_2.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5 && \
PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=/tmp/tune_v.json PDT_AUTOTUNE=0 run s4v_fresh_2.txt 400 python bench.py --model vit_b_16 --fp8 --steps 15 --warmup 5
