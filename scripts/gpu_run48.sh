source scripts/gpurun_lib.sh
run r48_pmc_a.log 120 timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD -d gpurun_out/pmc48a -o run --output-format csv -- python3 scripts/probe_linear_wgrad.py
run r48_pmc_b.log 120 timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc48b -o run --output-format csv -- python3 scripts/probe_linear_wgrad.py
exit 0
