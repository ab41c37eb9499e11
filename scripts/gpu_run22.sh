source scripts/gpurun_lib.sh
run r22_tests.txt 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider
run r22_bench_r50.txt 400 python bench.py --steps 30 --warmup 10
run r22_bench_vit.txt 500 python bench.py --model vit_b_16 --batch 256 --steps 10 --warmup 5
run r22_bench_vit8.txt 500 python bench.py --model vit_b_16 --fp8 --batch 256 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
run r22_bench_r152.txt 500 python bench.py --model resnet152 --batch 512 --steps 10 --warmup 5
cp pytorch_distributed_template_amd/_lib/autotune_gfx950.json gpurun_out/autotune_gfx950.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run r22_pmc_attn.log 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_attn22 -o run --output-format csv -- python3 scripts/attn_one.py
exit 0
