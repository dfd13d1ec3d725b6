# round 4 first GPU call: the whole -m gpu suite (distributed tests last), the default bench,
# then the watchdog probe (its case A is expected to abort a child process, so it runs last)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4_gpu_tests.log
[ $rc -eq 0 ] || { grep -B2 -A30 "^E \|FAILED\|Error" gpurun_out/r4_gpu_tests.log | tail -60; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { tail -30 gpurun_out/r4_bench.err; exit 1; }
tail -1 gpurun_out/r4_bench.json | cut -c1-300
timeout -k 10 400 python tools/watchdog_capture_probe.py > gpurun_out/r4_watchdog_probe.txt 2>&1
cat gpurun_out/r4_watchdog_probe.txt
