# same-box A/B of an environment knob on the default bench: bash tools/gpu_ab_env.sh VAR valA valB [bench args]
V=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out
for r in 1 2; do
  for val in "$A" "$B"; do
    env $V=$val timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 "$@" > gpurun_out/ab_env.json 2> gpurun_out/ab_env.err || { tail -20 gpurun_out/ab_env.err; exit 1; }
    python -c "import json;r=json.load(open('gpurun_out/ab_env.json'));print('$V=$val', round(r['ms_per_step'],3), 'ms', 'pbwd', round(r['roofline']['mean_us'],1))"
  done
done
