# round-3 measurement batch: outlier-injection parity + its train-step cost, 1-GPU kernel profile,
# captured union-step floor, emulated rank-of-8 with / without the point side on a second stream,
# fp32 vs bf16 camera projections (same tree)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_outliers.py > gpurun_out/t_outliers.log 2>&1
tail -1 gpurun_out/t_outliers.log
timeout -k 10 300 python tools/train_step_bench.py --steps 6 --outliers 0.1 > gpurun_out/tsb_out.log 2>&1
tail -4 gpurun_out/tsb_out.log | cut -c1-300
bash tools/prof_full.sh r3c > /dev/null
head -3 gpurun_out/pf_r3c_breakdown.txt
timeout -k 10 400 python tools/train_step_bench.py --steps 3 --capture-floor > gpurun_out/tsb_cap.log 2>&1 || true
grep capture gpurun_out/tsb_cap.log | cut -c1-300 || true
for v in 0 1; do
  GASFM_SIDE_STREAM=$v timeout -k 10 300 python bench.py --emulate-world 8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/em8_side$v.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/em8_side$v.json').read().strip().splitlines()[-1]);print('emulated rank 0 of 8, side stream $v:', round(d['ms_per_step'],3))"
done
for pr in fp32 bf16; do
  timeout -k 10 300 python bench.py --proj-precision $pr --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$pr.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/bench_$pr.json').read().strip().splitlines()[-1]);print('config 4 proj $pr:', round(d['ms_per_step'],3))"
done
