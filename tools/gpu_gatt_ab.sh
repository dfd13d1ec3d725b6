# Round 6: adaptive point chunk of the global attention (a rank's shard: 64-point chunks) -- tests, A/B
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_global_attn.py tests/test_gpu_global.py tests/test_distributed.py > gpurun_out/gatt_tests.log 2>&1 || { tail -30 gpurun_out/gatt_tests.log; exit 1; }
tail -1 gpurun_out/gatt_tests.log
for lib in libgasfm.so libgasfm_gatt0.so libgasfm.so libgasfm_gatt0.so; do
  GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/gatt_em8.json 2> gpurun_out/gatt_em8.err || { tail -20 gpurun_out/gatt_em8.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gatt_em8.json').read().strip().splitlines()[-1]);print('em8 $lib', round(d['ms_per_step'],3))"
done
GASFM_LIB=$PWD/gasfm_amd/libgasfm.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/gatt_c4.json 2> gpurun_out/gatt_c4.err || { tail -20 gpurun_out/gatt_c4.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/gatt_c4.json').read().strip().splitlines()[-1]);print('c4 new', round(d['ms_per_step'],3))"
for lib in libgasfm.so libgasfm_gatt0.so; do
  echo "== gatt_bench $lib"; GASFM_LIB=$PWD/gasfm_amd/$lib timeout -k 10 120 python tools/gatt_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
