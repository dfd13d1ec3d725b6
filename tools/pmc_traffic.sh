# HBM traffic of the fused attention forward from PMC counters (GPU box).
# Two passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), counters only, no traces;
# kernel-filtered to attn_fwd_kernel; a short bench run of the same workload.
set -e
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "attn_fwd" --output-format csv \
    -d $ROOT/gpurun_out/pmc_$C -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    > $ROOT/gpurun_out/pmc_$C.log 2>&1
done
cd $ROOT && python tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_attn_fwd.json && cp gpurun_out/pmc_attn_fwd.json profiles/r2_pmc_attn_fwd.json
