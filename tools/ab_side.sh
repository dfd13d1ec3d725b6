# A/B of the point-side side stream (streams.py): GPU tests, then config 4 and the 1/8 proxy with it on/off
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
for n in 200000 25000; do
  for s in 1 0; do
    GASFM_SIDE_STREAM=$s timeout -k 10 300 python bench.py --n $n --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_${n}_$s.log 2>gpurun_out/b_${n}_$s.err
    python -c "import json,sys;d=json.loads(open('gpurun_out/b_${n}_$s.log').read().strip().splitlines()[-1]);print('n=$n side=$s',d['ms_per_step'],d['execution'])"
  done
done
