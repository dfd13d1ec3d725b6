set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "point or node or model" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in libgasfm.so libgasfm_nored.so; do echo $v; GASFM_LIB=$PWD/gasfm_amd/$v timeout -k 10 100 python tools/point_bench.py 16 25000 200000 2>&1 | grep kernel; done
timeout -k 10 180 python tools/edge_bench.py > gpurun_out/eb.log 2>&1; grep node_ gpurun_out/eb.log
