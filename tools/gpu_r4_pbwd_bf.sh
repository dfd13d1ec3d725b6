# round 4: edge_cam_pbwd without exec-mask branches in its tile loop (GASFM_PBWD_BF=1 build,
# gasfm_amd/libgasfm_bf.so): its edge_cam parity tests, then the pbwd A/B against the default
set -o pipefail
mkdir -p gpurun_out
GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_cam.py -x -q --timeout 300 --timeout-method thread > gpurun_out/bf_tests.log 2>&1 || { tail -30 gpurun_out/bf_tests.log; exit 1; }
tail -1 gpurun_out/bf_tests.log
bash tools/gpu_pbwd_ab.sh "$@"
