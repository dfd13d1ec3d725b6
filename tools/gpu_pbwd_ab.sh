# folded edge_cam_pbwd A/B (round 3): the edge_cam parity tests on the default library, then per
# library (default + given variants) the pbwd launches alone (tools/edge_bench.py: base, EPI, DWP,
# EPI+DWP) and the config-4 bench with the fold, two rounds
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge_cam.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pbwd_tests.log 2>&1 || { tail -30 gpurun_out/pbwd_tests.log; exit 1; }
tail -1 gpurun_out/pbwd_tests.log
for rep in 1 2; do
for lib in libgasfm.so "$@"; do
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python tools/edge_bench.py --reps 10 > gpurun_out/pbwd_eb.log 2>/dev/null
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pbwd_bench.log 2>/dev/null
  python -c "
import json
eb=[json.loads(l) for l in open('gpurun_out/pbwd_eb.log') if l.startswith('{')]
pb=[(d['kernel'].split('(')[1].rstrip(')'), d['us']) for d in eb if d['kernel'].startswith('edge_cam_pbwd')]
d=json.loads(open('gpurun_out/pbwd_bench.log').read().strip().splitlines()[-1])
print('$lib'.ljust(20), pb, 'config4', round(d['ms_per_step'],3), 'ms')"
done
done
