# Round 6: the point tail + hub forward as one kernel (GASFM_TAIL_HUB) -- parity tests, then config 4 and the
# rank-0-of-8 proxy alternating with / without, then kernel traces of both
# (its kernel-trace step looked for a stats csv the default output format does not write; tools/gpu_tail_hub_prof.sh took the per-kernel times)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_point_block.py tests/test_gpu_model.py tests/test_gpu_train_step.py > gpurun_out/th_tests.log 2>&1 || { tail -30 gpurun_out/th_tests.log; exit 1; }
tail -1 gpurun_out/th_tests.log
for F in 1 0 1 0; do
  GASFM_TAIL_HUB=$F timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/th_em8.json 2> gpurun_out/th_em8.err || { tail -20 gpurun_out/th_em8.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/th_em8.json').read().strip().splitlines()[-1]);print('em8 tail_hub=$F', round(d['ms_per_step'],3))"
  GASFM_TAIL_HUB=$F timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/th_c4.json 2> gpurun_out/th_c4.err || { tail -20 gpurun_out/th_c4.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/th_c4.json').read().strip().splitlines()[-1]);print('config4 tail_hub=$F', round(d['ms_per_step'],3))"
done
cd /tmp && export TMPDIR=/tmp
for F in 1 0; do
  GASFM_TAIL_HUB=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/th_prof$F -o run -- python3 $GRAFT_REPO_ROOT/bench.py --emulate-world 8 --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/th_prof$F.log 2>&1 || exit 1
  GASFM_TAIL_HUB=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/th_c4prof$F -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/th_c4prof$F.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for F in 1 0; do
  echo "== proxy tail_hub=$F"; grep -E "point_(tail|hub)_(hub_)?fwd" gpurun_out/th_prof$F/run_kernel_stats.csv | cut -d, -f1-5
  echo "== config4 tail_hub=$F"; grep -E "point_(tail|hub)_(hub_)?fwd" gpurun_out/th_c4prof$F/run_kernel_stats.csv | cut -d, -f1-5
done
