#!/bin/bash
# Dump the counters rocprofv3 offers on this agent (names differ across ROCm releases).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
echo "[rc=$?]" >> gpurun_out/counters_list.txt
