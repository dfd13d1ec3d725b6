# global-chain GPU tests + config-4 / proxy / emulated benches
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_global.py tests/test_gpu_model.py tests/test_distributed.py tests/test_gpu_grad_hygiene.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tq.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/tq.log | tail -60; tail -5 gpurun_out/tq.log; exit 1; }
tail -1 gpurun_out/tq.log
for args in "--n 200000" "--n 25000" "--emulate-world 8"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bq_$tag.log 2>gpurun_out/bq_$tag.err || { tail -20 gpurun_out/bq_$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bq_$tag.log').read().strip().splitlines()[-1]);print('$args', round(d['ms_per_step'],3), d['execution'][:20])"
done
