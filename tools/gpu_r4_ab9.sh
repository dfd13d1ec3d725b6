# round 4: the grouped attention backward (GASFM_ATTN_GRP_BWD=1): its oracle tests, then config 4
# and the proxy against the direct-to-LDS backward, same box, and the kernel times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attn_dispatch.py tests/test_gpu_attention.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab9_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab9_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab9_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab9.json 2> gpurun_out/ab9.err || { tail -20 gpurun_out/ab9.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab9.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run grp_bwd GASFM_ATTN_GRP_BWD=1
  EXTRA="--emulate-world 8"
  run default
  run grp_bwd GASFM_ATTN_GRP_BWD=1
done
GASFM_ATTN_GRP_BWD=1 bash tools/prof_full.sh r4gbwd > gpurun_out/ab9_prof.txt 2>&1 || { tail -20 gpurun_out/ab9_prof.txt; exit 1; }
grep -i "attn_bwd" gpurun_out/pf_r4gbwd_stats.csv | cut -c1-100
