# Round 6: the camera-side fp32 GEMMs on rocBLAS (TORCH_BLAS_PREFER_HIPBLASLT=0) vs hipBLASLt (default), config 4
mkdir -p gpurun_out
for v in 1 0 1 0; do
  TORCH_BLAS_PREFER_HIPBLASLT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/blas_c4.json 2> gpurun_out/blas_c4.err || { tail -20 gpurun_out/blas_c4.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/blas_c4.json').read().strip().splitlines()[-1]);print('prefer_hipblaslt=$v', round(d['ms_per_step'],3))"
done
