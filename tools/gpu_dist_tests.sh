# the multi-process distributed GPU tests alone (gloo ranks on one GPU, RCCL one-rank capture);
# verbose and unbuffered so a hang names its test (the silence watchdog sees the progress)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_distributed.py -m gpu -x -v -s --timeout 240 --timeout-method thread "$@" 2>&1 | grep --line-buffered -v "hostname of the client\|amdgpu.ids\|Gloo\] Rank" | tee gpurun_out/dist_tests.log | grep --line-buffered "PASSED\|FAILED\|Error\|error\|Traceback\|^E \|Timeout\|passed\|failed"
