# round 4 final evidence on this tree: full -m gpu suite, smoke, the default bench (with the CPU
# baseline), a kernel trace of the bench, per-kernel PMC traffic (two counter passes), the
# rank-0-of-8 proxy and its breakdown.  Everything lands in gpurun_out/ as r4f_*.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_gpu_tests.log 2>&1 || { grep -B5 -A30 "^E \|FAILED" gpurun_out/r4f_gpu_tests.log | head -80; tail -3 gpurun_out/r4f_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r4f_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { tail -30 gpurun_out/r4f_smoke.log; exit 1; }
tail -1 gpurun_out/r4f_smoke.log
SECONDS=0; timeout -k 10 600 python bench.py > gpurun_out/r4f_bench_default.json 2> gpurun_out/r4f_bench_default.err || { tail -30 gpurun_out/r4f_bench_default.err; exit 1; }
tail -1 gpurun_out/r4f_bench_default.json | cut -c1-400
echo "bench wall: ${SECONDS}s"
bash tools/prof_full.sh r4f > gpurun_out/r4f_prof.txt 2>&1 || { tail -20 gpurun_out/r4f_prof.txt; exit 1; }
head -8 gpurun_out/pf_r4f_breakdown.txt
bash tools/pmc_kernels.sh "edge_cam_pbwd|edge_seam_fwd|attn_bwd|attn_fwd_grp|point_hub_bwd|point_tail_bwd|segment_rowsum|gatt" r4f > gpurun_out/r4f_pmc.txt 2>&1 || { tail -20 gpurun_out/r4f_pmc.txt; exit 1; }
cat gpurun_out/r4f_pmc.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --emulate-world 8 > gpurun_out/r4f_em8.json 2> gpurun_out/r4f_em8.err || { tail -20 gpurun_out/r4f_em8.err; exit 1; }
tail -1 gpurun_out/r4f_em8.json | cut -c1-200
bash tools/prof_emul.sh r4f8 --emulate-world 8
