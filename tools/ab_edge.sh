# A/B: edge microbench on the default library and each variant given as an argument
set -e
timeout -k 10 180 python tools/edge_bench.py > gpurun_out/eb_default.log 2>&1; grep kernel gpurun_out/eb_default.log
for v in "$@"; do
  GASFM_LIB=$PWD/gasfm_amd/$v timeout -k 10 180 python tools/edge_bench.py > gpurun_out/eb_$v.log 2>&1; grep kernel gpurun_out/eb_$v.log
done
