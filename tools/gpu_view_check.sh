# view-block kernels: parity tests, model tests, step times
set -e
timeout -k 10 600 python -m pytest tests/test_gpu_view_block.py tests/test_gpu_point_block.py tests/test_gpu_model.py -x -q > gpurun_out/t.log 2>&1 || { tail -60 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 400 python tools/step_overhead.py > gpurun_out/ovh.log 2>&1; grep "graph" gpurun_out/ovh.log
