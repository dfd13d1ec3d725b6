# full GPU suite (continues past failing tests, stops on a crash / timeout), then smoke
mkdir -p gpurun_out
timeout -k 10 540 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_tests.log
[ $rc -le 1 ] || exit $rc
grep -E "^(FAILED|ERROR)" gpurun_out/r6_tests.log | head -20
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || { tail -30 gpurun_out/r6_smoke.log; exit 1; }
tail -1 gpurun_out/r6_smoke.log
