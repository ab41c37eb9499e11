source scripts/gpurun_lib.sh
export PDT_AUTOTUNE_CACHE=$PWD/gpurun_out/tune_s4b.json
run s4b_op_on.txt 600 python -u scripts/op_profile.py --top 90 && \
run s4b_op_off.txt 600 python -u scripts/op_profile.py --top 90 --set PDT_FUSE_BN_AX1=0
