# Round 6: camera-direction piece length of a rank-of-8 shard (GASFM_MAX_PIECE) -- the proxy
mkdir -p gpurun_out
for P in ${PIECES:-64 48 64 48 64 48}; do
  if [ "$P" = 0 ]; then unset GASFM_MAX_PIECE; else export GASFM_MAX_PIECE=$P; fi; timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/piece_em8.json 2> gpurun_out/piece_em8.err || { tail -20 gpurun_out/piece_em8.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/piece_em8.json').read().strip().splitlines()[-1]);print('piece $P', round(d['ms_per_step'],3), 'pbwd', round(d['roofline']['mean_us'],1))"
done
