# A/B of library variants against the default (gasfm_amd/<name>.so): config 4 and the rank-0-of-8
# proxy, two rounds, same box
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for lib in libgasfm.so "$@"; do
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_c4.log 2>/dev/null
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_em8.log 2>/dev/null
  python -c "
import json
a=json.loads(open('gpurun_out/ab_c4.log').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/ab_em8.log').read().strip().splitlines()[-1])
print('$lib'.ljust(24), 'config 4', round(a['ms_per_step'],3), '  rank 0 of 8', round(b['ms_per_step'],3))"
done
done
