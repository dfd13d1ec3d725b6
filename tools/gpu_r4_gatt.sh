# round 4: parity of the fused global convs (global_attn.hip), then the same-box A/B and a trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_global_attn.py tests/test_gpu_global.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4g_tests.log
[ $rc -eq 0 ] || { grep -B2 -A25 "^E \|FAILED\|Error" gpurun_out/r4g_tests.log | head -80; exit $rc; }
for v in 1 0 1 0; do
  for args in "--emulate-world 8" ""; do
    GASFM_GLOBAL_ATTN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('gatt=$v', '$args', round(d['ms_per_step'],3))"
  done
done
bash tools/prof_emul.sh r4em8d --emulate-world 8
timeout -k 10 300 python tools/torch_prof.py --n 200000 --emulate-world 8 --stacks --rows 60 > gpurun_out/r4_torchprof_em8.txt 2>&1
