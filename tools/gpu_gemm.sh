# fp32 GEMM: parity of gasfm_gemm_f32 (new large-tile kernel), then the new vs the round-3 kernel vs hipBLASLt
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_f32.py -q -x --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/gemm_new.txt 2>&1 || { tail -20 gpurun_out/gemm_new.txt; exit 1; }
cat gpurun_out/gemm_new.txt
GASFM_GEMM_F32_OLD=1 timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/gemm_old.txt 2>&1 || { tail -20 gpurun_out/gemm_old.txt; exit 1; }
cat gpurun_out/gemm_old.txt
