# fp32 GEMM + view-chain GPU tests, then config 4 / proxy / emulated benches with the HIP GEMM and with hipBLASLt
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_f32.py tests/test_gpu_view_block.py tests/test_gpu_bf16_proj.py tests/test_gpu_model.py tests/test_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tgm.log 2>&1 || { grep -B5 "Error\|assert" gpurun_out/tgm.log | tail -60; tail -5 gpurun_out/tgm.log; exit 1; }
tail -1 gpurun_out/tgm.log
for gm in hip torch; do
for args in "--n 200000" "--emulate-world 8"; do
  tag=$(echo $gm$args | tr -d ' -')
  GASFM_VIEW_GEMM=$gm timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bg_$tag.log 2>gpurun_out/bg_$tag.err || { tail -20 gpurun_out/bg_$tag.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bg_$tag.log').read().strip().splitlines()[-1]);print('$gm $args', round(d['ms_per_step'],3), d['execution'][:20])"
done
done
