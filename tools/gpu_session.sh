# Session check: all GPU tests, smoke, default bench (with CPU baseline), rocprof kernel-trace --stats of the bench.
set -e
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
SECONDS=0; timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log; echo "bench wall: ${SECONDS}s"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_bench -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $ROOT/gpurun_out/prof_bench.log 2>&1
cd $ROOT && ls -R gpurun_out/prof_bench | head
python tools/step_breakdown.py gpurun_out/prof_bench/run_results.db 3 30 > gpurun_out/prof_bench_breakdown.txt
python tools/rocprof_summary.py gpurun_out/prof_bench/run_results.db gpurun_out/prof_bench_summary.csv 7 | tail -3
