# GEMM algorithm selection by torch's TunableOp (hipBLASLt + rocBLAS solutions timed per shape) for
# the hipBLASLt GEMMs of the config-4 step and its rank-0-of-8 proxy, then an A/B of both benches
# with and without the tuned table.  Usage: tools/tune_gemms.sh TAG (outputs gpurun_out/TAG_*).
TAG=${1:-tune}
set -o pipefail
mkdir -p gpurun_out
F=gpurun_out/${TAG}_tunableop.csv
export PYTORCH_TUNABLEOP_FILENAME=$F
B="--no-cpu-baseline"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 400 python bench.py --steps 2 --warmup 2 $B --eager > gpurun_out/${TAG}_t1.json 2> gpurun_out/${TAG}_t1.err || { tail -20 gpurun_out/${TAG}_t1.err; exit 1; }
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 400 python bench.py --steps 2 --warmup 2 $B --eager --emulate-world 8 > gpurun_out/${TAG}_t8.json 2> gpurun_out/${TAG}_t8.err || { tail -20 gpurun_out/${TAG}_t8.err; exit 1; }
ls gpurun_out | grep tunableop
wc -l gpurun_out/${TAG}_tunableop*.csv
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_base$r.json 2>/dev/null || exit 1
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_tuned$r.json 2> gpurun_out/${TAG}_tuned$r.err || { tail -20 gpurun_out/${TAG}_tuned$r.err; exit 1; }
  timeout -k 10 300 python bench.py $B --emulate-world 8 --steps 20 > gpurun_out/${TAG}_base8_$r.json 2>/dev/null || exit 1
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py $B --emulate-world 8 --steps 20 > gpurun_out/${TAG}_tuned8_$r.json 2>/dev/null || exit 1
  for k in base$r tuned$r base8_$r tuned8_$r; do echo "$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_$k.json)"; done
done
