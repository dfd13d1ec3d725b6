# round 4: same-box A/B of the fused global chain / view chain on the rank-0-of-8 proxy and config 4, then a trace
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  for args in "--emulate-world 8" ""; do
    GASFM_GLOBAL_CHAIN=$1 GASFM_VIEW_CHAIN=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('gchain=$1 vchain=$2', '$args', round(d['ms_per_step'],3))"
  done
done
done
bash tools/prof_emul.sh r4em8b --emulate-world 8
