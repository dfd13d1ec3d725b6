# round 4: the forward seam's items dealt XCD-contiguously (libgasfm_sx.so, GASFM_SEAM_XCD=1) vs the
# default: its tests, config 4 and the proxy, same box, then the seam's PMC traffic with the variant
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
GASFM_LIB=$PWD/gasfm_amd/libgasfm_sx.so timeout -k 10 400 $T tests/test_gpu_edge_cam.py > gpurun_out/ab13_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab13_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab13_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab13.json 2> gpurun_out/ab13.err || { tail -20 gpurun_out/ab13.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab13.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run seam_xcd GASFM_LIB=$PWD/gasfm_amd/libgasfm_sx.so
  EXTRA="--emulate-world 8"
  run default
  run seam_xcd GASFM_LIB=$PWD/gasfm_amd/libgasfm_sx.so
done
GASFM_LIB=$PWD/gasfm_amd/libgasfm_sx.so bash tools/prof_full.sh r4sx > gpurun_out/ab13_prof.txt 2>&1 || { tail -20 gpurun_out/ab13_prof.txt; exit 1; }
grep -i "seam" gpurun_out/pf_r4sx_stats.csv | cut -c1-140
GASFM_LIB=$PWD/gasfm_amd/libgasfm_sx.so bash tools/pmc_kernels.sh "edge_seam_fwd" r4sx > gpurun_out/ab13_pmc.txt 2>&1 || { tail -20 gpurun_out/ab13_pmc.txt; exit 1; }
cat gpurun_out/ab13_pmc.txt
