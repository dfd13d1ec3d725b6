# Block-0 kernels: the row-order prologue (GASFM_E0_ROWS) and the 4-group epilogue backward
# (libgasfm_u1.so = one row group per step): tests, same-box bench A/Bs, a kernel-trace profile.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_block.py tests/test_gpu_model.py tests/test_gpu_train_step.py tests/test_gpu_edge_cam.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e0_tests.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/e0_tests.log | tail -40; tail -5 gpurun_out/e0_tests.log; exit 1; }
tail -2 gpurun_out/e0_tests.log
b() { timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/e0_bench.log 2>/dev/null
      python -c "import json;d=json.loads(open('gpurun_out/e0_bench.log').read().strip().splitlines()[-1]);print('$1', round(d['ms_per_step'],3), 'ms/step')"; }
for rep in 1 2; do
  GASFM_E0_ROWS=0 GASFM_LIB=$PWD/gasfm_amd/libgasfm_u1.so b "old (scatter, U=1)"
  GASFM_LIB=$PWD/gasfm_amd/libgasfm_u1.so b "rows, U=1"
  b "rows, U=4 (default)"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e0 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_e0.log 2>&1
ls -R gpurun_out/prof_e0 | head -20
