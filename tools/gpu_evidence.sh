# Evidence batch on this tree: full -m gpu suite, smoke, the default bench (with the CPU baseline),
# a kernel trace of the bench, per-kernel PMC traffic (two counter passes), the rank-0-of-8 proxy
# and its breakdown.  Usage: tools/gpu_evidence.sh TAG (outputs in gpurun_out/ as TAG_*).
TAG=${1:-ev}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { grep -B5 -A30 "^E \|FAILED" gpurun_out/${TAG}_gpu_tests.log | head -80; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
SECONDS=0; timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { tail -30 gpurun_out/${TAG}_bench_default.err; exit 1; }
tail -1 gpurun_out/${TAG}_bench_default.json | cut -c1-400
echo "bench wall: ${SECONDS}s"
bash tools/prof_full.sh ${TAG} > gpurun_out/${TAG}_prof.txt 2>&1 || { tail -20 gpurun_out/${TAG}_prof.txt; exit 1; }
head -8 gpurun_out/pf_${TAG}_breakdown.txt
bash tools/pmc_kernels.sh "edge_cam_pbwd|edge_seam_fwd|attn_bwd|attn_fwd_grp|point_hub_bwd|point_tail_bwd|segment_rowsum|gatt" ${TAG} > gpurun_out/${TAG}_pmc.txt 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.txt; exit 1; }
cat gpurun_out/${TAG}_pmc.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 > gpurun_out/${TAG}_em8.json 2> gpurun_out/${TAG}_em8.err || { tail -20 gpurun_out/${TAG}_em8.err; exit 1; }
tail -1 gpurun_out/${TAG}_em8.json | cut -c1-200
bash tools/prof_emul.sh ${TAG}8 --emulate-world 8
