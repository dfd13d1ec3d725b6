# forward-seam A/B (round 3): edge parity tests on the default library, then edge_seam_fwd alone
# (tools/edge_bench.py) and the config-4 bench for the default and each given variant, two rounds
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_block.py tests/test_gpu_edge_cam.py -x -q --timeout 120 --timeout-method thread > gpurun_out/seam_tests.log 2>&1 || { tail -30 gpurun_out/seam_tests.log; exit 1; }
tail -2 gpurun_out/seam_tests.log
for rep in 1 2; do
for lib in libgasfm.so "$@"; do
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python tools/edge_bench.py --reps 20 > gpurun_out/seam_eb.log 2>/dev/null
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/seam_bench.log 2>/dev/null
  python -c "
import json
eb=[json.loads(l) for l in open('gpurun_out/seam_eb.log') if l.startswith('{')]
seam=[d for d in eb if 'seam' in json.dumps(d)]
d=json.loads(open('gpurun_out/seam_bench.log').read().strip().splitlines()[-1])
print('$lib'.ljust(20), 'seam', [round(x.get('us', 0), 1) for x in seam], 'config4', round(d['ms_per_step'],3), 'ms')"
done
done
