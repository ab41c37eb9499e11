source scripts/gpurun_lib.sh
run r40_prof_vit.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit_40 -o run --output-format csv -- python3 bench.py --model vit_b_16 --batch 256 --steps 4 --warmup 3
run r40_prof_vit8.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit8_40 -o run --output-format csv -- python3 bench.py --model vit_b_16 --fp8 --batch 256 --steps 4 --warmup 3
exit 0
