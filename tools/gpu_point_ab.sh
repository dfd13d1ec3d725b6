# point-kernel A/B: tail / hub parity tests on the default library, then tools/point_bench.py for each
# library variant given (gasfm_amd/<name>.so)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_point_block.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_tests.log 2>&1 || { tail -30 gpurun_out/pt_tests.log; exit 1; }
tail -2 gpurun_out/pt_tests.log
for lib in libgasfm.so "$@"; do
  echo "== $lib"
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 120 python tools/point_bench.py 2>&1 | grep "kernel us"
done
