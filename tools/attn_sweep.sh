# Wave-cap sweep of the attention kernels (one process per setting: the cap is read once).
set -e
for w in default 4096 7168 14336 28672 57344 1000000; do
  if [ "$w" = default ]; then unset GASFM_ATTN_WAVES; else export GASFM_ATTN_WAVES=$w; fi
  timeout -k 10 120 python tools/attn_bench.py --reps 20 >> gpurun_out/sweep.log 2>&1
done
cat gpurun_out/sweep.log | grep direction
