# round 4: SQ stall counters of the step's largest kernels on the final tree (one counter pass)
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_sq.sh "edge_cam_pbwd|edge_seam_fwd|point_hub_bwd|point_tail_bwd|attn_bwd_glds|attn_fwd_grp" r4f bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4_sq.txt 2>&1 || { tail -20 gpurun_out/r4_sq.txt; exit 1; }
cat gpurun_out/r4_sq.txt
