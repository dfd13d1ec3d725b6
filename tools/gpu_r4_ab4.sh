# round 4: the 256-thread combine (libgasfm_cmb.so, GASFM_COMBINE_SMALL=1) and 32-edge camera
# pieces on the rank-0-of-8 proxy against the default, same box; config 2's captured step on this
# tree; an op-level profile of the proxy.  DXL: the GASFM_DXL_PT setting to run with.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
GASFM_LIB=$PWD/gasfm_amd/libgasfm_cmb.so timeout -k 10 300 $T tests/test_gpu_attention.py tests/test_gpu_attn_dispatch.py > gpurun_out/ab4_tests_cmb.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab4_tests_cmb.log | head -60; exit 1; }
tail -1 gpurun_out/ab4_tests_cmb.log
run() {
  local label=$1; shift
  env GASFM_DXL_PT=${DXL:-0} "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab4.json 2> gpurun_out/ab4.err || { tail -20 gpurun_out/ab4.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab4.json').read().strip().splitlines()[-1]);print('$label'.ljust(24), '$EXTRA'.ljust(20), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  EXTRA=""
  run default
  run cmb GASFM_LIB=$PWD/gasfm_amd/libgasfm_cmb.so
  EXTRA="--emulate-world 8"
  run default
  run cmb GASFM_LIB=$PWD/gasfm_amd/libgasfm_cmb.so
  run piece32 GASFM_MAX_PIECE=32
  run cmb,piece32 GASFM_LIB=$PWD/gasfm_amd/libgasfm_cmb.so GASFM_MAX_PIECE=32
done
GASFM_DXL_PT=${DXL:-0} timeout -k 10 300 python tools/single_scene_bench.py --steps 50 --warmup 3 > gpurun_out/r4_config2.jsonl 2> gpurun_out/r4_config2.err || { tail -20 gpurun_out/r4_config2.err; exit 1; }
cat gpurun_out/r4_config2.jsonl
GASFM_DXL_PT=${DXL:-0} timeout -k 10 300 python tools/torch_prof.py --n 200000 --emulate-world 8 --stacks --rows 80 > gpurun_out/r4_torchprof_em8.txt 2>&1 || tail -5 gpurun_out/r4_torchprof_em8.txt
