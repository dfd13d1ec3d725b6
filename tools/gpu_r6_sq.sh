# Round 6 final tree: SQ counters of the step's big kernels (config 4), one counter-only pass
mkdir -p gpurun_out
bash tools/pmc_sq.sh "edge_cam_pbwd|edge_seam_fwd|point_hub_bwd_r|point_tail_bwd_r|attn_fwd_grp|attn_bwd_glds|segment_rowsum" r6final bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r6_sq_table.txt 2>&1 || { tail -20 gpurun_out/r6_sq_table.txt; tail -20 gpurun_out/sq_r6final.log; exit 1; }
cat gpurun_out/r6_sq_table.txt
