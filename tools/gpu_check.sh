# GPU box: parity tests, a bench line, and a kernel-trace profile of the bench (rocpd db -> csv).
set -e
OUT=${1:-prof}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -3 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b.log 2>&1 && tail -1 gpurun_out/b.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/p.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py gpurun_out/$OUT/run_results.db gpurun_out/$OUT/kernel_stats.csv 7
