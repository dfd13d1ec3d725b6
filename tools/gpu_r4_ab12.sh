# round 4: edge_cam_pbwd with fewer registers held across tiles (GASFM_PBWD_DB_LDS=1: the camera bias
# sums in LDS; =2: also the LayerNorm affine re-read per tile; =3: also the softmax constants) vs the default, same box
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
GASFM_LIB=$PWD/gasfm_amd/libgasfm_db3.so timeout -k 10 400 $T tests/test_gpu_edge_cam.py > gpurun_out/ab12_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab12_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab12_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab12.json 2> gpurun_out/ab12.err || { tail -20 gpurun_out/ab12.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab12.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3), 'pbwd_us', round(r.get('mean_us') or 0,1))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run db1 GASFM_LIB=$PWD/gasfm_amd/libgasfm_db1.so
  run db2 GASFM_LIB=$PWD/gasfm_amd/libgasfm_db2.so
  run db3 GASFM_LIB=$PWD/gasfm_amd/libgasfm_db3.so
  EXTRA="--emulate-world 8"
  run default
  run db2 GASFM_LIB=$PWD/gasfm_amd/libgasfm_db2.so
  run db3 GASFM_LIB=$PWD/gasfm_amd/libgasfm_db3.so
done
