#!/bin/bash
# Per-shape native vs MIOpen conv kernels at the bench batch (2048), MIOpen's find db seeded
# from the bs-2048 ResNet-50 runs (profiles/miopen_db_bs2048) so no cold find runs.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/miopen_db
cp -n profiles/miopen_db_bs2048/*.txt gpurun_out/miopen_db/ 2>/dev/null || true
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 900 python -u scripts/bench_kernels.py --batch 2048 > gpurun_out/conv_kernels_native_vs_miopen_bs2048.txt 2>&1
