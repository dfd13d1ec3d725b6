# Round 6: PyTorch TunableOp over the step's torch GEMMs (the camera-side fp32 products on hipBLASLt):
# tune once in eager mode (every GEMM shape of the config-4 step), then A/B the captured bench reading the results
mkdir -p gpurun_out
rm -f gpurun_out/tunableop_results*.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 \
PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_results.csv \
  timeout -k 10 500 python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tune.json 2> gpurun_out/tune.err || { tail -30 gpurun_out/tune.err; exit 1; }
ls -la gpurun_out/ | grep tunableop
f=$(ls gpurun_out/tunableop_results*.csv | head -1); echo "results: $f"; wc -l "$f"; head -30 "$f"
for v in 0 1 0 1; do
  PYTORCH_TUNABLEOP_ENABLED=$v PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/$f \
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/tuned_c4.json 2> gpurun_out/tuned_c4.err || { tail -20 gpurun_out/tuned_c4.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/tuned_c4.json').read().strip().splitlines()[-1]);print('tunableop=$v', round(d['ms_per_step'],3), d['execution'][:40])"
done
