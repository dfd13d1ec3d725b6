# all GPU tests, edge microbench, config-4 / per-rank-proxy graph step times
set -e
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 180 python tools/edge_bench.py > gpurun_out/eb.log 2>&1; grep kernel gpurun_out/eb.log
timeout -k 10 400 python tools/step_overhead.py > gpurun_out/ovh.log 2>&1; grep "graph" gpurun_out/ovh.log
