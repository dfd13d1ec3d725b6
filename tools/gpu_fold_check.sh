# epilogue-fold check (round 3): the edge_cam / edge-block parity tests, then edge_cam_pbwd alone
# (tools/edge_bench.py) and the config-4 bench with GASFM_EPI_FOLD=0 / 1, two rounds
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_cam.py tests/test_gpu_edge_block.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/fold_tests.log 2>&1 || { tail -40 gpurun_out/fold_tests.log; exit 1; }
grep -E "passed|failed|launches" gpurun_out/fold_tests.log | tail -4
for rep in 1 2; do
for f in 0 1; do
  GASFM_EPI_FOLD=$f timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fold_bench.log 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/fold_bench.log').read().strip().splitlines()[-1]);print('EPI_FOLD=$f', round(d['ms_per_step'],3), 'ms/step', round(d['value']/1e6,1), 'M edges/s', 'pbwd', round(d['roofline']['mean_us'],1))"
done
done
