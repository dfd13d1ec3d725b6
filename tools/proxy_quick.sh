# graph-mode step time at config 4 and at the per-rank size of an 8-GPU run
set -e
timeout -k 10 400 python tools/step_overhead.py > gpurun_out/ovh.log 2>&1; grep "graph" gpurun_out/ovh.log
