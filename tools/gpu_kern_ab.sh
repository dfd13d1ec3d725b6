# kernel-level A/B: tools/edge_bench.py (edge, camera-fused, point kernels at config-4 sizes) for the
# default library and each variant given (gasfm_amd/<name>.so), two rounds, one line per kernel
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for lib in libgasfm.so "$@"; do
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 240 python tools/edge_bench.py --reps 20 > gpurun_out/kab_$lib.log 2>&1 || { tail -20 gpurun_out/kab_$lib.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/kab_$lib.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$lib'.ljust(22), d['kernel'].ljust(28), d['us'], d['GBps'])
"
done
done
