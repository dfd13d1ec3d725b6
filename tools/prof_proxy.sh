# kernel trace of the 1/8-points proxy (the per-rank load of an 8-GPU run), graph replay
# usage: bash tools/prof_proxy.sh [extra bench args...]
set -e
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/prof_proxy -o run -- python3 $ROOT/bench.py --n 25000 --steps 5 --warmup 2 --no-cpu-baseline "$@" > $ROOT/gpurun_out/pp.log 2>&1
cd $ROOT && tail -1 gpurun_out/pp.log | cut -c1-400 && python tools/step_breakdown.py gpurun_out/prof_proxy/run_results.db 4 60
