# rank-0-of-8 proxy and config 4 at fixed camera-direction piece lengths vs the size-aware default
set -e
mkdir -p gpurun_out
for mp in default 256; do
  if [ $mp = default ]; then unset GASFM_MAX_PIECE; else export GASFM_MAX_PIECE=$mp; fi
  timeout -k 10 300 python bench.py --emulate-world 8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/em8_mp$mp.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/em8_mp$mp.json').read().strip().splitlines()[-1]);print('emulated rank 0 of 8, max_piece $mp:', round(d['ms_per_step'],3))"
done
unset GASFM_MAX_PIECE
