# A/B of an environment setting (e.g. GASFM_L1_THRESHOLD=128) on config 4 and the 1/8 proxy, 2 rounds
set -e
for rep in 1 2; do
  for e in "X=0" "$1"; do
    for n in 200000 25000; do
      env $e timeout -k 10 300 python bench.py --points $n --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ae_$n.log 2>/dev/null
      python -c "import json;d=json.loads(open('gpurun_out/ae_$n.log').read().strip().splitlines()[-1]);print('$e n=$n', round(d['ms_per_step'],3))"
    done
  done
done
