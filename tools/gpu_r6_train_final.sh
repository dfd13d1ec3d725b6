# the B = 1 training steps (configs 3 / 5, captured + pipelined) and the sharded config-5 proxy on the final tree
mkdir -p gpurun_out
timeout -k 10 200 python tools/train_step_bench.py --batch 1 --captured --pipeline --gasfm-adam --no-eager --steps 30 --prime 40 --progress 5 > gpurun_out/r6f_ts_b1_c3.jsonl 2> gpurun_out/r6f_ts_b1_c3.err || { tail -30 gpurun_out/r6f_ts_b1_c3.err; exit 1; }
cat gpurun_out/r6f_ts_b1_c3.jsonl
timeout -k 10 200 python tools/train_step_bench.py --batch 1 --outliers 0.1 --captured --pipeline --gasfm-adam --no-eager --steps 30 --prime 60 --progress 5 > gpurun_out/r6f_ts_b1_c5.jsonl 2> gpurun_out/r6f_ts_b1_c5.err || { tail -30 gpurun_out/r6f_ts_b1_c5.err; exit 1; }
cat gpurun_out/r6f_ts_b1_c5.jsonl
timeout -k 10 180 python tools/dist_train_bench.py --emulate-world 8 --steps 20 > gpurun_out/r6f_dt_em8.json 2> gpurun_out/r6f_dt_em8.err || { tail -30 gpurun_out/r6f_dt_em8.err; exit 1; }
cat gpurun_out/r6f_dt_em8.json
