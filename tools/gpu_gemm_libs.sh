# gemm_bench at m = 1000 for library variants: bash tools/gpu_gemm_libs.sh lib...
for lib in libgasfm.so "$@"; do
  echo "== $lib"
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 120 python tools/gemm_bench.py 2>/dev/null | grep "m= 1000" || exit 1
done
