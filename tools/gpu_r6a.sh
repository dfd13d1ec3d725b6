# Round 6 first pass: full GPU suite (continues past failing tests, stops on a crash / timeout),
# smoke, default bench, rank-0-of-8 proxy, the B = 1 training steps (configs 3 / 5, captured +
# pipelined), the sharded config-5 step's proxy.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6a_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6a_tests.log
[ $rc -le 1 ] || exit $rc
grep -E "^(FAILED|ERROR)" gpurun_out/r6a_tests.log | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a_smoke.log 2>&1 || { tail -30 gpurun_out/r6a_smoke.log; exit 1; }
tail -1 gpurun_out/r6a_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || { tail -30 gpurun_out/r6a_bench.err; exit 1; }
tail -1 gpurun_out/r6a_bench.json
timeout -k 10 300 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/r6a_em8.json 2> gpurun_out/r6a_em8.err || { tail -30 gpurun_out/r6a_em8.err; exit 1; }
tail -1 gpurun_out/r6a_em8.json
timeout -k 10 400 python tools/train_step_bench.py --batch 1 --captured --pipeline --gasfm-adam --no-eager --steps 30 --prime 40 > gpurun_out/r6a_ts_b1_c3.jsonl 2> gpurun_out/r6a_ts_b1_c3.err || { tail -30 gpurun_out/r6a_ts_b1_c3.err; exit 1; }
cat gpurun_out/r6a_ts_b1_c3.jsonl
timeout -k 10 400 python tools/train_step_bench.py --batch 1 --outliers 0.1 --captured --pipeline --gasfm-adam --no-eager --steps 30 --prime 60 > gpurun_out/r6a_ts_b1_c5.jsonl 2> gpurun_out/r6a_ts_b1_c5.err || { tail -30 gpurun_out/r6a_ts_b1_c5.err; exit 1; }
cat gpurun_out/r6a_ts_b1_c5.jsonl
timeout -k 10 300 python tools/dist_train_bench.py --emulate-world 8 --steps 20 > gpurun_out/r6a_dt_em8.json 2> gpurun_out/r6a_dt_em8.err || { tail -30 gpurun_out/r6a_dt_em8.err; exit 1; }
cat gpurun_out/r6a_dt_em8.json
GASFM_WGRAD_GEMM=torch timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r6a_bench_wgrad_torch.json 2> gpurun_out/r6a_bench_wgrad_torch.err || { tail -30 gpurun_out/r6a_bench_wgrad_torch.err; exit 1; }
tail -1 gpurun_out/r6a_bench_wgrad_torch.json
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r6a_bench_wgrad_hip.json 2> gpurun_out/r6a_bench_wgrad_hip.err || { tail -30 gpurun_out/r6a_bench_wgrad_hip.err; exit 1; }
tail -1 gpurun_out/r6a_bench_wgrad_hip.json
