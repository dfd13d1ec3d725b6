# Full GPU suite + smoke + default bench (tools/gpu_full.sh), then the edge0_epilogue_bwd A/B
# (libgasfm_u1.so = one row group per step) and a kernel-trace profile of the default bench.
set -e
mkdir -p gpurun_out
bash tools/gpu_full.sh
b() { timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/e0_bench.log 2>/dev/null
      python -c "import json;d=json.loads(open('gpurun_out/e0_bench.log').read().strip().splitlines()[-1]);print('$1', round(d['ms_per_step'],3), 'ms/step')"; }
for rep in 1 2; do
  GASFM_LIB=$PWD/gasfm_amd/libgasfm_u1.so b "U=1"
  b "U=4 (default)"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e0f -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_e0f.log 2>&1
echo profiled
