# round 4: the fused global convs with whole chunks requested at once (this tree) against the
# previous version (libgasfm_gprev.so), and the mask-only branch-free pbwd (libgasfm_bf1.so,
# GASFM_PBWD_BF=1), same box
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_global_attn.py tests/test_gpu_global.py > gpurun_out/ab8_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab8_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab8_tests.log
GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf1.so timeout -k 10 300 $T tests/test_gpu_edge_cam.py > gpurun_out/ab8_tests_bf1.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab8_tests_bf1.log | head -60; exit 1; }
tail -1 gpurun_out/ab8_tests_bf1.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab8.json 2> gpurun_out/ab8.err || { tail -20 gpurun_out/ab8.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab8.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3), 'pbwd_us', round(r.get('mean_us') or 0,1))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run gprev GASFM_LIB=$PWD/gasfm_amd/libgasfm_gprev.so
  run pbwd_bf1 GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf1.so
  EXTRA="--emulate-world 8"
  run default
  run gprev GASFM_LIB=$PWD/gasfm_amd/libgasfm_gprev.so
done
bash tools/prof_full.sh r4gatt2 > gpurun_out/ab8_prof.txt 2>&1 || { tail -20 gpurun_out/ab8_prof.txt; exit 1; }
grep -i "gatt" gpurun_out/pf_r4gatt2_stats.csv | cut -c1-120
