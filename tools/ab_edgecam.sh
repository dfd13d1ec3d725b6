# A/B of the fused edge prologue + camera attention (GASFM_EDGE_CAM) on the config-4 bench, same box,
# then a kernel trace of the fused step.
set -e
mkdir -p gpurun_out
for v in 1 0 1; do
  GASFM_EDGE_CAM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_ec$v.json 2> gpurun_out/ab_ec$v.err
  python -c "import json; r=json.load(open('gpurun_out/ab_ec$v.json')); print('EDGE_CAM=$v', round(r['ms_per_step'],3), 'ms', round(r['value']/1e6,1), 'M edges/s')"
done
bash tools/prof_full.sh ec "$@"
