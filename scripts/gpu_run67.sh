source scripts/gpurun_lib.sh
run r67_prof_vit.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r67_vit -o run --output-format csv -- python3 bench.py --model vit_b_16 --steps 4 --warmup 3
run r67_prof_vit_fp8.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r67_vitf8 -o run --output-format csv -- python3 bench.py --model vit_b_16 --fp8 --steps 4 --warmup 3
exit 0
