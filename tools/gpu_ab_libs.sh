# Library / knob A/B (round 5): parity tests of the edge kernels on the default library, then per
# variant -- the default, then each argument: a library gasfm_amd/<name>.so or an environment
# assignment VAR=value (default library) -- the edge kernels alone at config-4 size
# (tools/edge_bench.py: seam, pbwd EPI+DWP) and the config-4 and rank-0-of-8 benches, two rounds.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_edge_cam.py tests/test_gpu_model.py tests/test_gpu_attention.py tests/test_gpu_global_attn.py tests/test_gpu_point_block.py tests/test_gpu_view_block.py tests/test_gpu_edge_block.py > gpurun_out/ab_tests.log 2>&1 || { grep -B5 -A30 "^E \|FAILED" gpurun_out/ab_tests.log | head -80; exit 1; }
tail -1 gpurun_out/ab_tests.log
for rep in 1 2; do
for lib in libgasfm.so "$@"; do
  envs=(GASFM_LIB=$PWD/gasfm_amd/$lib)
  case "$lib" in *=*) envs=(GASFM_LIB=$PWD/gasfm_amd/libgasfm.so "$lib");; esac
  env "${envs[@]}" timeout -k 10 300 python tools/edge_bench.py --reps 10 > gpurun_out/ab_eb.log 2>/dev/null
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_c4.json 2>/dev/null || { echo "bench failed $lib"; exit 1; }
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 > gpurun_out/ab_em8.json 2>/dev/null || { echo "em8 failed $lib"; exit 1; }
  python - "$lib" <<'PY'
import json, sys
eb = [json.loads(l) for l in open("gpurun_out/ab_eb.log") if l.startswith("{")]
ks = {d["kernel"]: d["us"] for d in eb}
pick = {k: v for k, v in ks.items() if k.startswith(("edge_seam_fwd", "edge_cam_pbwd(LN, RES, EPI+DWP)", "edge_cam_fwd"))}
a = json.loads(open("gpurun_out/ab_c4.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/ab_em8.json").read().strip().splitlines()[-1])
r = a.get("roofline") or {}
print(sys.argv[1].ljust(24), "c4", round(a["ms_per_step"], 3), "em8", round(b["ms_per_step"], 3),
      "pbwd_us", round(r.get("mean_us") or 0, 1), pick, flush=True)
PY
done
done
