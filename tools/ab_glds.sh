# A/B of the direct-to-LDS attention forward (GASFM_ATTN_GLDS)
set -e
timeout -k 10 120 python tools/attn_bench.py --reps 20 > gpurun_out/ab0.log 2>&1; grep direction gpurun_out/ab0.log
GASFM_ATTN_GLDS=0 timeout -k 10 120 python tools/attn_bench.py --reps 20 > gpurun_out/ab1.log 2>&1; grep direction gpurun_out/ab1.log
timeout -k 10 600 python -m pytest tests/test_gpu_attention.py tests/test_gpu_model.py tests/test_gpu_edge_block.py tests/test_distributed.py -x -q > gpurun_out/tg.log 2>&1 || { tail -30 gpurun_out/tg.log; exit 1; }
tail -1 gpurun_out/tg.log
