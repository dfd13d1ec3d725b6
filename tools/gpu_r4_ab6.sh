# round 4: the full -m gpu parity suite on this tree, the default bench and the rank-0-of-8 proxy
# with the measured defaults, config 2's captured step, an op-level profile of the proxy
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1 || { grep -B5 -A30 "^E \|FAILED" gpurun_out/r4_gpu_tests.log | head -80; tail -3 gpurun_out/r4_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4_gpu_tests.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab6_c4.json 2> gpurun_out/ab6.err || { tail -20 gpurun_out/ab6.err; exit 1; }
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 > gpurun_out/ab6_em8.json 2> gpurun_out/ab6.err || { tail -20 gpurun_out/ab6.err; exit 1; }
  python -c "
import json
a=json.loads(open('gpurun_out/ab6_c4.json').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/ab6_em8.json').read().strip().splitlines()[-1])
print('config 4', round(a['ms_per_step'],3), 'ms', round(a['value']/1e6,1), 'M edges/s   rank 0 of 8', round(b['ms_per_step'],3))"
done
timeout -k 10 300 python tools/single_scene_bench.py --steps 50 --warmup 3 > gpurun_out/r4_config2.jsonl 2> gpurun_out/r4_config2.err || { tail -20 gpurun_out/r4_config2.err; exit 1; }
cat gpurun_out/r4_config2.jsonl
timeout -k 10 300 python tools/torch_prof.py --n 200000 --emulate-world 8 --stacks --rows 80 > gpurun_out/r4_torchprof_em8.txt 2>&1 || tail -5 gpurun_out/r4_torchprof_em8.txt
bash tools/prof_emul.sh r4em8f --emulate-world 8
