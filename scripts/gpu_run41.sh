source scripts/gpurun_lib.sh
run r41_avail.txt 60 rocprofv3 -L
run r41_pmc_a.log 90 timeout -s KILL 80 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc41a -o run --output-format csv -- python3 scripts/conv_one.py 256 14 256 3 1 fwd
run r41_pmc_b.log 90 timeout -s KILL 80 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc41b -o run --output-format csv -- python3 scripts/conv_one.py 64 56 64 3 1 fwd
run r41_pmc_c.log 90 timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc41c -o run --output-format csv -- python3 scripts/conv_one.py 256 14 256 3 1 fwd
exit 0
