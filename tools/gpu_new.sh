# Run a subset of GPU tests (args = pytest targets), log to gpurun_out/tnew.log.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/tnew.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/tnew.log | tail -80; tail -5 gpurun_out/tnew.log; exit 1; }
tail -3 gpurun_out/tnew.log
