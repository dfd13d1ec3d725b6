# Round 6 final tree: kernel trace of the config-4 bench (graph replay): stats csv, one-step breakdown, attention per
# direction (the trace database stays in /tmp; only the summaries come back)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_c4f -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/pf_c4f.log 2>&1
cd $R
tail -1 gpurun_out/pf_c4f.log | cut -c1-300
python tools/rocprof_summary.py /tmp/prof_c4f/run_results.db gpurun_out/pf_c4f_stats.csv 5 > /dev/null
python tools/step_breakdown.py /tmp/prof_c4f/run_results.db 4 40 > gpurun_out/pf_c4f_breakdown.txt
python tools/attn_direction_stats.py /tmp/prof_c4f/run_results.db > gpurun_out/pf_c4f_attn_dirs.txt
head -12 gpurun_out/pf_c4f_breakdown.txt
