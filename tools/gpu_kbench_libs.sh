# per-kernel microbenchmarks (attention, point kernels) for library variants: bash tools/gpu_kbench_libs.sh lib...
mkdir -p gpurun_out
for lib in libgasfm.so "$@"; do
  echo "== $lib"
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 200 python tools/attn_bench.py --reps 10 2>/dev/null | cut -c1-220 || exit 1
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 200 python tools/point_bench.py 2>/dev/null | cut -c1-220 || exit 1
done
