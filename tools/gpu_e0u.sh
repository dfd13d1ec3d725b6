# edge0_epilogue_bwd row groups per step: default (U=1) vs libgasfm_u2.so / libgasfm_u4.so, same box,
# then a kernel-trace profile of the default bench.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_block.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e0_tests.log 2>&1 || { tail -30 gpurun_out/e0_tests.log; exit 1; }
tail -1 gpurun_out/e0_tests.log
b() { timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/e0_bench.log 2>/dev/null
      python -c "import json;d=json.loads(open('gpurun_out/e0_bench.log').read().strip().splitlines()[-1]);print('$1', round(d['ms_per_step'],3), 'ms/step')"; }
for rep in 1 2; do
  b "U=1 (default)"
  GASFM_LIB=$PWD/gasfm_amd/libgasfm_u2.so b "U=2"
  GASFM_LIB=$PWD/gasfm_amd/libgasfm_u4.so b "U=4"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e0u -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_e0u.log 2>&1
echo profiled
