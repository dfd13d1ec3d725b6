# Bench-argument A/B (round 5): per variant -- each argument is a string of extra bench.py
# arguments, "" for the default -- the config-4 and rank-0-of-8 benches, two rounds, one line each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for args in "$@"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/ab_c4.json 2>/dev/null || { echo "bench failed: $args"; exit 1; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 $args > gpurun_out/ab_em8.json 2>/dev/null || { echo "em8 failed: $args"; exit 1; }
  python - "$args" <<'PY'
import json, sys
a = json.loads(open("gpurun_out/ab_c4.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/ab_em8.json").read().strip().splitlines()[-1])
print(repr(sys.argv[1]).ljust(28), "c4", round(a["ms_per_step"], 3), "em8", round(b["ms_per_step"], 3), flush=True)
PY
done
done
