# torch's BLAS backend for the camera-side GEMMs: hipBLASLt (default) vs rocBLAS, config 4 and the
# rank-0-of-8 proxy, two rounds on one box
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for pref in 1 0; do
  TORCH_BLAS_PREFER_HIPBLASLT=$pref timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bl_c4.log 2>/dev/null
  TORCH_BLAS_PREFER_HIPBLASLT=$pref timeout -k 10 300 python bench.py --emulate-world 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bl_em8.log 2>/dev/null
  python -c "
import json
a=json.loads(open('gpurun_out/bl_c4.log').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/bl_em8.log').read().strip().splitlines()[-1])
print('TORCH_BLAS_PREFER_HIPBLASLT=$pref', 'config 4', round(a['ms_per_step'],3), '  rank 0 of 8', round(b['ms_per_step'],3))"
done
done
