# round 4: the camera side's weight-gradient GEMMs on a second stream (GASFM_SIDE_GEMM=1) vs one
# stream: the bitwise test, then config 4, same box
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_model.py -k "side_gemm or side_stream" > gpurun_out/ab15_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab15_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab15_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab15.json 2> gpurun_out/ab15.err || { tail -20 gpurun_out/ab15.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab15.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3))"
}
for rep in 1 2 3; do
  EXTRA=""
  run default
  run side_gemm GASFM_SIDE_GEMM=1
done
GASFM_SIDE_GEMM=1 bash tools/prof_full.sh r4sg > gpurun_out/ab15_prof.txt 2>&1 || { tail -20 gpurun_out/ab15_prof.txt; exit 1; }
head -6 gpurun_out/pf_r4sg_breakdown.txt
