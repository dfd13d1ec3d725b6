# edge-kernel A/B: edge parity tests on the default library, then the config-4 bench (graph replay)
# for the default and each given library variant (gasfm_amd/<name>.so), two rounds
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_block.py tests/test_gpu_edge_cam.py -x -q --timeout 120 --timeout-method thread > gpurun_out/edge_tests.log 2>&1 || { tail -30 gpurun_out/edge_tests.log; exit 1; }
tail -2 gpurun_out/edge_tests.log
for rep in 1 2; do
for lib in libgasfm.so "$@"; do
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench.log 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1]);print('$lib', round(d['ms_per_step'],3), 'ms/step', 'roofline', round(d['roofline']['frac'],3))"
done
done
