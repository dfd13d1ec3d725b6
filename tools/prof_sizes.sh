# kernel traces of graph-replayed steps at a tiny scene (fixed costs) and at the 1/8 proxy
set -e
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for n in 2000 25000; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/prof_n$n -o run -- python3 $ROOT/bench.py --n $n --steps 5 --warmup 2 --no-cpu-baseline > $ROOT/gpurun_out/prof_n$n.log 2>&1
  tail -1 $ROOT/gpurun_out/prof_n$n.log | cut -c1-200
done
