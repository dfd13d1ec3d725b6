# kernel trace of the config-4 bench (graph replay), stats csv + one-step breakdown + attention per direction
# usage: bash tools/prof_full.sh <tag> [extra bench args...]
set -e
ROOT=$GRAFT_REPO_ROOT
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_$TAG -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $ROOT/gpurun_out/pf_$TAG.log 2>&1
cd $ROOT
tail -1 gpurun_out/pf_$TAG.log | cut -c1-300
python tools/rocprof_summary.py gpurun_out/prof_$TAG/run_results.db gpurun_out/pf_${TAG}_stats.csv 5 > /dev/null
python tools/step_breakdown.py gpurun_out/prof_$TAG/run_results.db 4 40 > gpurun_out/pf_${TAG}_breakdown.txt
python tools/attn_direction_stats.py gpurun_out/prof_$TAG/run_results.db > gpurun_out/pf_${TAG}_attn_dirs.txt
head -30 gpurun_out/pf_${TAG}_breakdown.txt
cat gpurun_out/pf_${TAG}_attn_dirs.txt
