# round 4: the fused global convs with the two-level merge: parity, then forced on (GASFM_GLOBAL_ATTN=1)
# against the default (on for <= 64k point sources only) on config 4 and the proxy; the mask-only
# branch-free pbwd (libgasfm_bf1.so, GASFM_PBWD_BF=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_global_attn.py tests/test_gpu_global.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab7_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab7_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab7_tests.log
GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_cam.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab7_tests_bf1.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab7_tests_bf1.log | head -60; exit 1; }
tail -1 gpurun_out/ab7_tests_bf1.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab7.json 2> gpurun_out/ab7.err || { tail -20 gpurun_out/ab7.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab7.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run gatt_on GASFM_GLOBAL_ATTN=1
  run gatt_off GASFM_GLOBAL_ATTN=0
  run pbwd_bf1 GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf1.so
  EXTRA="--emulate-world 8"
  run default
  run gatt_off GASFM_GLOBAL_ATTN=0
done
GASFM_GLOBAL_ATTN=1 bash tools/prof_full.sh r4gatt > gpurun_out/ab7_prof.txt 2>&1 || { tail -20 gpurun_out/ab7_prof.txt; exit 1; }
grep -i "gatt" gpurun_out/pf_r4gatt_stats.csv | cut -c1-120
