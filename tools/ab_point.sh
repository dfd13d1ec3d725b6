# A/B: point kernel microbench on the default library and each variant given as an argument
set -e
timeout -k 10 180 python tools/point_bench.py > gpurun_out/pb_default.log 2>&1; grep kernel gpurun_out/pb_default.log
for v in "$@"; do
  echo "variant $v"
  GASFM_LIB=$PWD/gasfm_amd/$v timeout -k 10 180 python tools/point_bench.py > gpurun_out/pb_$v.log 2>&1; grep kernel gpurun_out/pb_$v.log
done
