# Given GPU test files/-k selection only: python -u pytest with per-test timeouts, log to gpurun_out/tsel.log
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > gpurun_out/tsel.log 2>&1 || { grep -B8 "Error\|assert" gpurun_out/tsel.log | tail -80; tail -5 gpurun_out/tsel.log; exit 1; }
grep -c PASSED gpurun_out/tsel.log; tail -1 gpurun_out/tsel.log
