# block-0 point-direction attention backward A/B (round 3): the attention parity tests with the
# lane-group kernel forced on, then one kernel-trace profile per setting (general kernel / G lanes
# per item) and the per-kernel lines of the block-0 backward
set -e
mkdir -p gpurun_out
GASFM_ATTN_BWD_LANES=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_attn_dispatch.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lanes_tests.log 2>&1 || { grep -E "Error|assert" gpurun_out/lanes_tests.log | head -20; tail -3 gpurun_out/lanes_tests.log; exit 1; }
tail -1 gpurun_out/lanes_tests.log
for v in 0 1; do
  GASFM_ATTN_BWD_LANES=$v bash tools/prof_full.sh lanes$v > /dev/null
  echo "GASFM_ATTN_BWD_LANES=$v: $(head -1 gpurun_out/pf_lanes${v}_breakdown.txt)"
  grep -E "attn_bwd_lanes|attn_bwd_kernel<gasfm::Geom<4, 1>" gpurun_out/pf_lanes${v}_breakdown.txt || true
done
