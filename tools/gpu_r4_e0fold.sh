# round 4: block 0's epilogue backward folded into block 1's edge_cam_pbwd (GASFM_E0_FOLD): its tests,
# then config 4 and the proxy against edge0_epilogue_bwd, same box, and the kernel times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_cam.py -x -q --timeout 300 --timeout-method thread > gpurun_out/e0f_tests.log 2>&1 || { grep -B2 -A40 "^E \|FAILED\|Error" gpurun_out/e0f_tests.log | head -80; exit 1; }
tail -1 gpurun_out/e0f_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/e0f.json 2> gpurun_out/e0f.err || { tail -20 gpurun_out/e0f.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/e0f.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  EXTRA=""
  run fold
  run nofold GASFM_E0_FOLD=0
  EXTRA="--emulate-world 8"
  run fold
  run nofold GASFM_E0_FOLD=0
done
bash tools/prof_full.sh r4e0f > gpurun_out/e0f_prof.txt 2>&1 || { tail -20 gpurun_out/e0f_prof.txt; exit 1; }
grep -i "pbwd\|edge0_epi" gpurun_out/pf_r4e0f_stats.csv | cut -c1-140
