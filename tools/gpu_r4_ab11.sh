# round 4: the point side on a second stream (GASFM_SIDE_STREAM=1) re-measured on the round-4 kernels
# (config 4 and the rank-0-of-8 proxy, same box), after its bitwise test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k side_stream -x -q --timeout 200 --timeout-method thread > gpurun_out/ab11_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab11_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab11_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab11.json 2> gpurun_out/ab11.err || { tail -20 gpurun_out/ab11.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab11.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), '$EXTRA'.ljust(18), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run side GASFM_SIDE_STREAM=1
  EXTRA="--emulate-world 8"
  run default
  run side GASFM_SIDE_STREAM=1
done
