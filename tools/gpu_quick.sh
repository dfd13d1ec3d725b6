set -e
timeout -k 10 120 python tools/attn_bench.py --reps 20 > gpurun_out/ab.log 2>&1; cat gpurun_out/ab.log | grep direction
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b.log 2>&1 && tail -1 gpurun_out/b.log
