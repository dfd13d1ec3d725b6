# round 4: parity of the fused global convs, the point-ordered dXL path, the LDS-staged seam, the
# grouped segment row sums (+ the branch-free pbwd build), then same-box A/Bs on config 4 (20
# replayed steps, 2 alternations) and the rank-0-of-8 proxy, then a kernel trace of the proxy.
# libgasfm.so = this tree, libgasfm_bf.so = this tree with GASFM_PBWD_BF=1.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_global_attn.py tests/test_gpu_global.py tests/test_gpu_edge_cam.py tests/test_gpu_edge_block.py > gpurun_out/ab3_tests.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab3_tests.log | head -60; exit 1; }
tail -1 gpurun_out/ab3_tests.log
GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf.so timeout -k 10 300 $T tests/test_gpu_edge_cam.py > gpurun_out/ab3_tests_bf.log 2>&1 || { grep -B2 -A30 "^E \|FAILED" gpurun_out/ab3_tests_bf.log | head -60; exit 1; }
tail -1 gpurun_out/ab3_tests_bf.log
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/ab3.json 2> gpurun_out/ab3.err || { tail -20 gpurun_out/ab3.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab3.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$label'.ljust(28), '$EXTRA'.ljust(18), round(d['ms_per_step'],3), 'pbwd_us', round(r.get('mean_us') or 0,1))"
}
ALL="GASFM_DXL_PT=1 GASFM_SEAM_LDS=1 GASFM_ROWSUM_GRP=1"
for rep in 1 2; do
  EXTRA=""
  run default
  run dxl GASFM_DXL_PT=1
  run seam_lds GASFM_SEAM_LDS=1
  run rowsum_grp GASFM_ROWSUM_GRP=1
  run bf GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf.so
  run all $ALL
  run all+bf $ALL GASFM_LIB=$PWD/gasfm_amd/libgasfm_bf.so
  run gatt0 GASFM_GLOBAL_ATTN=0
done
for rep in 1 2; do
  EXTRA="--emulate-world 8"
  run default
  run all $ALL
  run gatt0 GASFM_GLOBAL_ATTN=0
done
env $ALL bash tools/prof_emul.sh r4em8e --emulate-world 8
