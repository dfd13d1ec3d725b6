# epilogue-fold A/B (round 3): config-4 bench with GASFM_EPI_FOLD=0 / 1 on the default library and
# GASFM_EPI_FOLD=1 on each given variant (gasfm_amd/<name>.so), two rounds; pbwd = the folded
# edge_cam_pbwd's mean launch time (bench.py roofline.mean_us)
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "0 libgasfm.so" "1 libgasfm.so" $(for l in "$@"; do echo "1:$l"; done); do
  f=${cfg%%[ :]*}; lib=${cfg##*[ :]}
  GASFM_LIB=$PWD/gasfm_amd/$lib GASFM_EPI_FOLD=$f timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fold_bench.log 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/fold_bench.log').read().strip().splitlines()[-1]);print('EPI_FOLD=$f $lib', round(d['ms_per_step'],3), 'ms/step', round(d['value']/1e6,1), 'M edges/s', 'pbwd', round(d['roofline']['mean_us'],1))"
done
done
