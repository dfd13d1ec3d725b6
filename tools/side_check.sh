set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_reduce.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ts.log 2>&1 || { grep -B5 "Error\|differ\|passed\|failed" gpurun_out/ts.log | tail -30; exit 1; }
tail -2 gpurun_out/ts.log
PYTHONPATH=. timeout -k 10 200 python tools/side_probe.py --capture-first 2>&1 | grep -v Warn | tail -4
