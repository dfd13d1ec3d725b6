# round 4: parity of the fused chains, then the same-box A/B and a trace of the proxy
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_global.py tests/test_gpu_view_block.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_tests.log
[ $rc -eq 0 ] || { grep -B2 -A25 "^E \|FAILED\|Error" gpurun_out/r4c_tests.log | head -80; exit $rc; }
for v in "1 1" "0 0" "1 1" "0 0"; do
  set -- $v
  for args in "--emulate-world 8" ""; do
    GASFM_GLOBAL_CHAIN=$1 GASFM_VIEW_CHAIN=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('gchain=$1 vchain=$2', '$args', round(d['ms_per_step'],3))"
  done
done
bash tools/prof_emul.sh r4em8c --emulate-world 8
