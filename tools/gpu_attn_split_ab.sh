# Round 6: lane groups per item (GASFM_ATTN_SPLIT) of the grouped point-direction forward, kernel alone at a
# rank-of-8 shard's size and at config 4, then the rank-0-of-8 proxy step per setting (same box)
mkdir -p gpurun_out
for P in 25000 200000; do for S in 1 2 4; do
  r=$(GASFM_ATTN_SPLIT=$S timeout -k 10 120 python tools/attn_bench.py --points $P 2>/dev/null | grep "segment order") || exit 1
  echo "points $P split $S $r"
done; done
for S in 1 2 4 1 2 4; do
  GASFM_ATTN_SPLIT=$S timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/split_em8.json 2> gpurun_out/split_em8.err || { tail -20 gpurun_out/split_em8.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/split_em8.json').read().strip().splitlines()[-1]); a=d['roofline_attention']; print('em8 split $S', round(d['ms_per_step'],3), 'attn_us', round(a['mean_us'],2), 'frac', round(a['frac'],3))"
done
