set -o pipefail
for rep in 1 2; do
for v in "" "GASFM_MAX_PIECE=128" "GASFM_MAX_PIECE=96"; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 > gpurun_out/ab_em8.json 2>/dev/null || { echo "em8 failed $v"; exit 1; }
  python -c "import json;b=json.loads(open('gpurun_out/ab_em8.json').read().strip().splitlines()[-1]);print('$v'.ljust(24),'em8',round(b['ms_per_step'],3))"
done
done
