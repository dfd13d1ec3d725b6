# full GPU suite + smoke, then the rank-0-of-8 proxy and the default bench (round 6, after a kernel change)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6s_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6s_tests.log
[ $rc -le 1 ] || exit $rc
grep -E "^(FAILED|ERROR)" gpurun_out/r6s_tests.log | head -20
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s_smoke.log 2>&1 || { tail -30 gpurun_out/r6s_smoke.log; exit 1; }
tail -1 gpurun_out/r6s_smoke.log
timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/r6s_em8.json 2> gpurun_out/r6s_em8.err || { tail -30 gpurun_out/r6s_em8.err; exit 1; }
tail -1 gpurun_out/r6s_em8.json | cut -c1-300
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r6s_bench.json 2> gpurun_out/r6s_bench.err || { tail -30 gpurun_out/r6s_bench.err; exit 1; }
tail -1 gpurun_out/r6s_bench.json | cut -c1-300
