source scripts/gpurun_lib.sh
run r51_bench_a.txt 400 python bench.py
run r51_bench_b.txt 400 python bench.py
cp gpurun_out/r50_autotune_gfx950.json pytorch_distributed_template_amd/_lib/autotune_gfx950.json
run r51_bench_c.txt 400 python bench.py
run r51_bench_d.txt 400 python bench.py
exit 0
