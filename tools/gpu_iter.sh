# Iteration check: GPU tests (optionally a -k filter in $1), then config-4 bench and the 1/8-points proxy.
set -e
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
fi
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b.log 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python -c "import json; r=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print('config4 ms/step', round(r['ms_per_step'],2), 'edges/s %.4g' % r['value'], 'attn frac', round(r['roofline']['frac'],3))"
timeout -k 10 300 python bench.py --n 25000 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp.log 2> gpurun_out/bp.err || { tail -20 gpurun_out/bp.err; exit 1; }
python -c "import json; r=json.loads(open('gpurun_out/bp.log').read().strip().splitlines()[-1]); print('proxy n=25k ms/step', round(r['ms_per_step'],2))"
