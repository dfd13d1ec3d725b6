# attention microbench + the attention parity tests only
set -e
timeout -k 10 120 python tools/attn_bench.py --reps 20 > gpurun_out/ab.log 2>&1; grep direction gpurun_out/ab.log
timeout -k 10 600 python -m pytest tests/test_gpu_attention.py -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
