# GPU tests of the given files, then config 4 and the 1/8 proxy bench (graph replay)
set -e
timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/tf.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/tf.log | tail -40; exit 1; }
tail -1 gpurun_out/tf.log
for n in 200000 25000; do
  timeout -k 10 300 python bench.py --points $n --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bf_$n.log 2>gpurun_out/bf_$n.err || { tail -20 gpurun_out/bf_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bf_$n.log').read().strip().splitlines()[-1]);print('n=$n', round(d['ms_per_step'],3), d['execution'][:20], 'frac', round(d['roofline']['frac'],3))"
done
