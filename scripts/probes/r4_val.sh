#!/bin/bash
# Round 4 validation: whole GPU suite, smoke, bench (driver defaults).
source "$(dirname "$0")/../gpurun_lib.sh"
T=${1:-r4v}
bash scripts/gpu_job.sh $T tests smoke bench
