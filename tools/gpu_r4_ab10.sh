# round 4: PyTorch TunableOp for the camera-side hipBLASLt GEMMs at one GPU (m = 1000 rows): one
# tuning pass (during the bench's warm-up, eager), then the tuned solutions (TUNING=0) against the
# default heuristics on config 4, same box.  The results file lands in gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_r4.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 500 python bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/ab10_tune.json 2> gpurun_out/ab10_tune.err || { tail -20 gpurun_out/ab10_tune.err; exit 1; }
ls gpurun_out/ | grep -i tunable
F=$(ls gpurun_out/tunableop_r4*.csv | head -1); echo "results: $F"; wc -l $F
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab10.json 2> gpurun_out/ab10.err || { tail -20 gpurun_out/ab10.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab10.json').read().strip().splitlines()[-1]);print('$label'.ljust(20), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  run default PYTORCH_TUNABLEOP_ENABLED=0
  run tunableop PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/$F
done
