# Round 6: the 48-edge camera pieces of a shard -- the sharded parity tests, the proxy
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_distributed.py tests/test_dist_train.py tests/test_gpu_edge_cam.py > gpurun_out/piece_tests.log 2>&1 || { tail -30 gpurun_out/piece_tests.log; exit 1; }
tail -1 gpurun_out/piece_tests.log
PIECES="0 0" bash tools/gpu_piece_ab.sh
