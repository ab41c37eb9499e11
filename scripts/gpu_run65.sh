source scripts/gpurun_lib.sh
L=pytorch_distributed_template_amd/_lib/libpdt_hip.so
for k in 1 2 3; do
  cp abtest/old.so $L && run r65_old_$k.txt 300 python bench.py
  cp abtest/new.so $L && run r65_new_$k.txt 300 python bench.py
done
exit 0
