# Round 6 final tree: the rank-0-of-8 proxy (bench line + rocprof breakdown) and the default bench
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/r6f_em8.json 2> gpurun_out/r6f_em8.err || { tail -30 gpurun_out/r6f_em8.err; exit 1; }
tail -1 gpurun_out/r6f_em8.json | cut -c1-300
bash tools/prof_emul.sh r6finalem8b --emulate-world 8
timeout -k 10 400 python bench.py > gpurun_out/r6f_bench.json 2> gpurun_out/r6f_bench.err || { tail -30 gpurun_out/r6f_bench.err; exit 1; }
tail -1 gpurun_out/r6f_bench.json | cut -c1-300
