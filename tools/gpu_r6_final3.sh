# Round 6 final tree after the fused point forward: rank-0-of-8 proxy (bench line + rocprof breakdown), default bench
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/r6f3_em8.json 2> gpurun_out/r6f3_em8.err || { tail -30 gpurun_out/r6f3_em8.err; exit 1; }
tail -1 gpurun_out/r6f3_em8.json | cut -c1-200
bash tools/prof_emul.sh r6f3em8 --emulate-world 8 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r6f3_bench.json 2> gpurun_out/r6f3_bench.err || { tail -30 gpurun_out/r6f3_bench.err; exit 1; }
tail -1 gpurun_out/r6f3_bench.json | cut -c1-200
