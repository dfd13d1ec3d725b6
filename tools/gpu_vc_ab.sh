# Round 6: the view chain's hub forward / first backward kernels at two workgroups per CU -- tests, proxy A/B
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_view_block.py tests/test_distributed.py > gpurun_out/vc_tests.log 2>&1 || { tail -30 gpurun_out/vc_tests.log; exit 1; }
tail -1 gpurun_out/vc_tests.log
for lib in libgasfm.so libgasfm_vc1.so libgasfm.so libgasfm_vc1.so libgasfm.so libgasfm_vc1.so; do
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/vc_em8.json 2> gpurun_out/vc_em8.err || { tail -20 gpurun_out/vc_em8.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/vc_em8.json').read().strip().splitlines()[-1]);print('em8 $lib', round(d['ms_per_step'],3))"
done
