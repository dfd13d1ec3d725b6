# round 4: the fused global convs with 8-view / 256-point chunks and batched merges (GASFM_GLOBAL_ATTN=1),
# grouped segment row sums, the 256-thread combine (libgasfm_cmb.so) and 32-edge camera
# pieces against the default (fused global convs now off), same box; then kernel traces of the
# default config-4 step and of the LDS-staged seam (GASFM_SEAM_LDS=1).
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_edge_block.py tests/test_gpu_global_attn.py > gpurun_out/ab5_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab5_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab5_tests.log
GASFM_LIB=$PWD/gasfm_amd/libgasfm_cmb.so timeout -k 10 300 $T tests/test_gpu_attention.py tests/test_gpu_attn_dispatch.py > gpurun_out/ab5_tests_cmb.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab5_tests_cmb.log | head -60; exit 1; }
tail -1 gpurun_out/ab5_tests_cmb.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab5.json 2> gpurun_out/ab5.err || { tail -20 gpurun_out/ab5.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab5.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run rowsum_grp GASFM_ROWSUM_GRP=1
  run cmb GASFM_LIB=$PWD/gasfm_amd/libgasfm_cmb.so
  run gatt1 GASFM_GLOBAL_ATTN=1
  EXTRA="--emulate-world 8"
  run default
  run gatt1 GASFM_GLOBAL_ATTN=1
  run rowsum_grp GASFM_ROWSUM_GRP=1
  run cmb GASFM_LIB=$PWD/gasfm_amd/libgasfm_cmb.so
  run piece32 GASFM_MAX_PIECE=32
done
bash tools/prof_full.sh r4def > gpurun_out/ab5_prof_def.txt 2>&1 || { tail -20 gpurun_out/ab5_prof_def.txt; exit 1; }
head -12 gpurun_out/pf_r4def_breakdown.txt
GASFM_SEAM_LDS=1 bash tools/prof_full.sh r4seam > gpurun_out/ab5_prof_seam.txt 2>&1 || { tail -20 gpurun_out/ab5_prof_seam.txt; exit 1; }
grep -i "seam" gpurun_out/pf_r4def_stats.csv gpurun_out/pf_r4seam_stats.csv | cut -c1-160
