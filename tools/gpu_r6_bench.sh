# default bench (with the CPU baseline), the rank-0-of-8 proxy, and the wgrad GEMM A/B
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err || { tail -30 gpurun_out/r6_bench.err; exit 1; }
tail -1 gpurun_out/r6_bench.json
timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/r6_em8.json 2> gpurun_out/r6_em8.err || { tail -30 gpurun_out/r6_em8.err; exit 1; }
tail -1 gpurun_out/r6_em8.json
GASFM_WGRAD_GEMM=torch timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r6_bench_wgrad_torch.json 2> gpurun_out/r6_bench_wgrad_torch.err || { tail -30 gpurun_out/r6_bench_wgrad_torch.err; exit 1; }
tail -1 gpurun_out/r6_bench_wgrad_torch.json
