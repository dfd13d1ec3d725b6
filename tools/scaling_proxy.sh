# per-rank load of an 8-GPU run on one GPU: eager vs hipGraph step, config 4 and 1/8 of its points
set -e
timeout -k 10 400 python tools/step_overhead.py > gpurun_out/ovh.log 2>&1; grep "n=" gpurun_out/ovh.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b.log 2>&1; tail -1 gpurun_out/b.log
