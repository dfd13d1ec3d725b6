# A/B of library variants (and env settings) on the config-4 bench step: entries are
# "lib[:VAR=val,...]"; 2 rounds, 10 timed steps each
set -e
for rep in 1 2; do
for spec in "$@"; do
  lib=${spec%%:*}; envs=""
  [[ "$spec" == *:* ]] && envs=$(echo "${spec#*:}" | tr ',' ' ')
  env GASFM_LIB=$PWD/gasfm_amd/$lib $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print('$spec', round(d['ms_per_step'],3), 'attn_fwd_pt_us', round(d['roofline']['mean_us'],1), 'frac', round(d['roofline']['frac'],3))"
done
done
