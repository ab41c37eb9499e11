# counter passes over scripts/attn_f8_one.py (fp8 attention fwd + fused bwd, ViT-B/16 bs1024)
source scripts/gpurun_lib.sh
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"
run attn_pmc1.txt 120 timeout -s KILL 100 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/attn_pmc1 -o run -- python3 scripts/attn_f8_one.py && \
run attn_pmc2.txt 120 timeout -s KILL 100 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/attn_pmc2 -o run -- python3 scripts/attn_f8_one.py && \
run attn_ktrace.txt 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attn_kt -o run -- python3 scripts/attn_f8_one.py && \
run attn_tests.txt 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "attention or vit"
