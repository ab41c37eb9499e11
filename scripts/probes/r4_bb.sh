#!/bin/bash
# Round 4: PyTorch TunableOp over the library (hipBLASLt) fp8 GEMMs of ViT-B/16 fp8 bs1024:
# tune once into gpurun_out/tunableop_vit.csv, then A/B with the tuned file (read only).
source "$(dirname "$0")/../gpurun_lib.sh"
T=r4bb
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=200 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_vit%d.csv run ${T}_tune.txt 900 python bench.py --model vit_b_16 --fp8 --steps 3 --warmup 2 || exit $?
ls -la gpurun_out/tunableop_vit* >> gpurun_out/${T}_tune.txt
for i in 1 2; do
run ${T}_vit_off$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_vit%d.csv run ${T}_vit_on$i.txt 400 python bench.py --model vit_b_16 --fp8 || exit $?
done
