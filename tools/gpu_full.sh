# Full GPU parity suite, smoke, then the default bench line (what the driver runs at round end).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/tg.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/tg.log | tail -60; tail -5 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
SECONDS=0; timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.log
echo "bench wall: ${SECONDS}s"
