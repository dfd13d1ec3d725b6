# env-switch A/B: the given GPU tests, then the config-4 bench with ENV=0 and ENV=1, two rounds
# usage: bash tools/gpu_env_ab.sh <ENV_NAME> <test files...>
set -e
mkdir -p gpurun_out
ENVN=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/envab_tests.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/envab_tests.log | tail -40; tail -5 gpurun_out/envab_tests.log; exit 1; }
  tail -2 gpurun_out/envab_tests.log
fi
for rep in 1 2; do
for v in 0 1; do
  env $ENVN=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/envab_bench.log 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/envab_bench.log').read().strip().splitlines()[-1]);print('$ENVN=$v', round(d['ms_per_step'],3), 'ms/step')"
done
done
