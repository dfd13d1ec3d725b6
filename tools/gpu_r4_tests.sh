# round 4: the full -m gpu suite and smoke on this tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t_gpu_tests.log 2>&1 || { grep -B5 -A30 "^E \|FAILED" gpurun_out/r4t_gpu_tests.log | head -80; tail -3 gpurun_out/r4t_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4t_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4t_smoke.log 2>&1 || { tail -30 gpurun_out/r4t_smoke.log; exit 1; }
tail -1 gpurun_out/r4t_smoke.log
