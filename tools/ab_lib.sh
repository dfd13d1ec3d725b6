# A/B of a library variant against the default: edge microbench, then config 4 and the 1/8 proxy (2 rounds)
set -e
V=$1
for lib in libgasfm.so $V; do
  echo "== $lib"; GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 200 python tools/edge_bench.py 2>&1 | grep -i "epilogue_fwd\|prologue_bwd" | head -4
done
for rep in 1 2; do
for lib in libgasfm.so $V; do
  for n in 200000 25000; do
    GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python bench.py --points $n --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$n.log 2>/dev/null
    python -c "import json;d=json.loads(open('gpurun_out/ab_$n.log').read().strip().splitlines()[-1]);print('$lib n=$n', round(d['ms_per_step'],3))"
  done
done
done
