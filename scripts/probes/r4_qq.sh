#!/bin/bash
# Round 4: fc2 data gradient with the act-3 epilogue (q11,cs key): tile 10 (tuned) vs tile 9.
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4qq
echo '{"f8b:201728,3072,768,1,3,0,q11,cs": 9}' > gpurun_out/tune_v9_r4qq.json
for i in 1 2; do
run ${T}_vit_v10_$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
PDT_AUTOTUNE_CACHE=gpurun_out/tune_v9_r4qq.json run ${T}_vit_v9_$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
