# round 4: XLc kept by the forward seam and read by edge_cam_pbwd (GASFM_XLC_STORE=1) vs the
# recompute: its test, then config 4 and the proxy, same box, and both kernels' times
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_edge_cam.py -k "xlc or fold or seam" > gpurun_out/ab16_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab16_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab16_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab16.json 2> gpurun_out/ab16.err || { tail -20 gpurun_out/ab16.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab16.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3), 'pbwd_us', round(r.get('mean_us') or 0,1))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run xlc_store GASFM_XLC_STORE=1
  EXTRA="--emulate-world 8"
  run default
  run xlc_store GASFM_XLC_STORE=1
done
GASFM_XLC_STORE=1 bash tools/prof_full.sh r4xs > gpurun_out/ab16_prof.txt 2>&1 || { tail -20 gpurun_out/ab16_prof.txt; exit 1; }
grep -i "pbwd\|seam" gpurun_out/pf_r4xs_stats.csv | cut -c1-130
