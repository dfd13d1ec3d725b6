# round 4: static priority 1 for the second-dispatched half of the resident grid (a CU's second
# workgroup) in edge_cam_pbwd (libgasfm_prio_p.so) and in edge_cam_pbwd + edge_seam_fwd
# (libgasfm_prio.so) vs the default, same box
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
GASFM_LIB=$PWD/gasfm_amd/libgasfm_prio.so timeout -k 10 400 $T tests/test_gpu_edge_cam.py > gpurun_out/ab14_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab14_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab14_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab14.json 2> gpurun_out/ab14.err || { tail -20 gpurun_out/ab14.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab14.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3), 'pbwd_us', round(r.get('mean_us') or 0,1))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run prio_pbwd GASFM_LIB=$PWD/gasfm_amd/libgasfm_prio_p.so
  run prio_both GASFM_LIB=$PWD/gasfm_amd/libgasfm_prio.so
  EXTRA="--emulate-world 8"
  run default
  run prio_both GASFM_LIB=$PWD/gasfm_amd/libgasfm_prio.so
done
