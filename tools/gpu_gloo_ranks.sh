# Round 6: bench.py's N-rank path at the driver's SCALE shapes, functionally (gloo, every rank on cuda:0): N = 4, 8
mkdir -p gpurun_out
for N in 4 8; do
  timeout -k 10 500 python bench.py --gpus $N --backend gloo --one-gpu --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gloo$N.json 2> gpurun_out/gloo$N.err || { tail -30 gpurun_out/gloo$N.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gloo$N.json').read().strip().splitlines()[-1]);print('N=$N n_gpus', d['n_gpus'], 'ms/step', round(d['ms_per_step'],1), d['config']['parallelism'][:80], '|', d['execution'][:60])"
done
