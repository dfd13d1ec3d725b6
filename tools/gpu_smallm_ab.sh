# small-M GEMM: parity tests, then the rank-0-of-8 proxy and the config-3 training step with the
# small-M kernels (GASFM_SMALLM_ROWS=256, default) and without (0), two rounds, same box
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_smallm.py tests/test_gpu_view_block.py tests/test_gpu_batch.py tests/test_distributed.py > gpurun_out/t_sm.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/t_sm.log | tail -40; tail -5 gpurun_out/t_sm.log; exit 1; }
tail -1 gpurun_out/t_sm.log
for rep in 1 2; do
for v in 256 0; do
  GASFM_SMALLM_ROWS=$v timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sm_em8.log 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/sm_em8.log').read().strip().splitlines()[-1]);print('GASFM_SMALLM_ROWS=$v rank 0 of 8', round(d['ms_per_step'],3))"
done
done
for v in 256 0; do
  GASFM_SMALLM_ROWS=$v timeout -k 10 300 python tools/train_step_bench.py --steps 6 --capture-floor > gpurun_out/sm_ts.log 2>&1
  grep -h "ms_replay\|ms_per_step" gpurun_out/sm_ts.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('GASFM_SMALLM_ROWS=$v', {k: round(v,2) for k,v in d.items() if k.startswith('ms')})"
done
