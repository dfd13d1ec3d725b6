# scene-build / outlier / batch / loss parity tests, then the config-3 and config-5 training-step
# benches, the rank-0-of-8 proxy and a short config-4 bench line
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_scene_device.py tests/test_gpu_outliers.py tests/test_gpu_batch.py tests/test_gpu_train_step.py tests/test_gpu_model.py tests/test_gpu_esfm_loss.py tests/test_distributed.py > gpurun_out/t_ts.log 2>&1 || { tail -30 gpurun_out/t_ts.log; exit 1; }
tail -1 gpurun_out/t_ts.log
timeout -k 10 300 python tools/train_step_bench.py --steps 6 > gpurun_out/tsb_c3.log 2>&1
grep ms_per_step gpurun_out/tsb_c3.log | cut -c1-400
timeout -k 10 300 python tools/train_step_bench.py --steps 6 --outliers 0.1 > gpurun_out/tsb_c5.log 2>&1
grep ms_per_step gpurun_out/tsb_c5.log | cut -c1-400
timeout -k 10 300 python bench.py --emulate-world 8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/em8.json 2>/dev/null
python -c "import json;d=json.loads(open('gpurun_out/em8.json').read().strip().splitlines()[-1]);print('emulated rank 0 of 8:', round(d['ms_per_step'],3))"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_rf.json 2> gpurun_out/bench_rf.err || { tail -20 gpurun_out/bench_rf.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_rf.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], json.dumps(d['roofline'])[:300])"
