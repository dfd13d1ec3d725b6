mkdir -p gpurun_out
for var in 6 10 11; do
  GASFM_GEMM_F32_VAR=$var timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_f32.py -q -x --timeout 120 --timeout-method thread > gpurun_out/gemm_tests_$var.log 2>&1 || { tail -30 gpurun_out/gemm_tests_$var.log; exit 1; }
  echo "var $var tests: $(tail -1 gpurun_out/gemm_tests_$var.log)"
done
for var in 6 10 11; do
  echo "var $var"
  GASFM_GEMM_F32_VAR=$var timeout -k 10 120 python tools/gemm_bench.py 2>/dev/null | grep "m= 1000" || exit 1
done
