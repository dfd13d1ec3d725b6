# distributed + view-chain GPU tests, then the per-rank proxies: the 1/8-points scene (all cameras, no
# sharding code) and rank 0 of an emulated 8-GPU step with points only / points + cameras sharded
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_distributed.py tests/test_gpu_view_block.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/td.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/td.log | tail -60; tail -5 gpurun_out/td.log; exit 1; }
tail -2 gpurun_out/td.log
for args in "--n 25000" "--emulate-world 8 --no-cam-shard" "--emulate-world 8"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bp_$tag.log 2>gpurun_out/bp_$tag.err || { tail -20 gpurun_out/bp_$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bp_$tag.log').read().strip().splitlines()[-1]);print('$args', round(d['ms_per_step'],3), d['execution'][:20])"
done
