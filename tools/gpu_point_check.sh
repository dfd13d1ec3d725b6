# point-block kernels: GPU parity tests + kernel microbench
set -e
timeout -k 10 600 python -m pytest tests/test_gpu_point_block.py tests/test_gpu_model.py -x -q > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 180 python tools/edge_bench.py > gpurun_out/eb.log 2>&1; grep -E "point|node" gpurun_out/eb.log
