# per-kernel durations of tools/point_bench.py (rocprofv3 kernel trace)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/hubprof -o run -- python3 $GRAFT_REPO_ROOT/tools/point_bench.py 25000 200000 > $GRAFT_REPO_ROOT/gpurun_out/hubprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/hubprof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/hubprof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | grep -i point
