# What the driver runs at round end: smoke, then the default bench (with the CPU baseline).
set -e
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
SECONDS=0; timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log
echo "bench wall: ${SECONDS}s"
