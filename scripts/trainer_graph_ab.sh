#!/bin/bash
# Trainer path (train.py, config/resnet50_bf16.json) with trainer.hip_graph off / on at one
# per-GPU batch: images/sec of the epoch from the Trainer's own meter.
#   gpurun -- bash scripts/trainer_graph_ab.sh TAG BATCH LEN_EPOCH
source "$(dirname "$0")/gpurun_lib.sh"
TAG=$1; BS=${2:-256}; LEN=${3:-60}
for G in false true; do
  python - <<PY
import json
c = json.load(open("config/resnet50_bf16.json"))
c["train_loader"]["args"]["batch_size"] = $BS
c["train_loader"]["args"]["num_samples"] = $BS * $LEN
c["trainer"].update(len_epoch=$LEN, epochs=2, save_dir="gpurun_out/${TAG}_ckpt", save_period=100, hip_graph=$( [ $G = true ] && echo True || echo False ))
json.dump(c, open("gpurun_out/${TAG}_cfg_$G.json", "w"))
PY
  PDT_RUN_ID=${TAG}_$G run ${TAG}_trainer_graph_$G.txt 600 python train.py -c gpurun_out/${TAG}_cfg_$G.json --no-validate || exit $?
  grep -h "images_per_sec" gpurun_out/${TAG}_trainer_graph_$G.txt
done
