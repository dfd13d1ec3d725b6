# round 4: global-chain kernels -- their parity tests + model tests, then config 4 and the rank-0-of-8 proxy
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_global.py tests/test_gpu_view_block.py tests/test_gpu_model.py tests/test_distributed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4c_tests.log
[ $rc -eq 0 ] || { grep -B2 -A25 "^E \|FAILED\|Error" gpurun_out/r4c_tests.log | head -80; exit $rc; }
for args in "" "--emulate-world 8"; do
  for chain in 1; do
    GASFM_GLOBAL_CHAIN=$chain timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/r4c_b.json 2> gpurun_out/r4c_b.err || { tail -20 gpurun_out/r4c_b.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r4c_b.json').read().strip().splitlines()[-1]);print('chain=$chain', '$args', round(d['ms_per_step'],3), d['execution'][:20])"
  done
done
