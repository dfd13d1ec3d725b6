# Round 6 (timing-only diagnostic): the point attention backward's per-item vmcnt(0) -- which also waits for the
# previous item's dXL stores -- vs a loose vmcnt(4) (libgasfm_loose.so; results not checked, timing only)
mkdir -p gpurun_out
for L in libgasfm.so libgasfm_loose.so libgasfm.so libgasfm_loose.so; do
  for P in 200000 25000; do
    r=$(GASFM_LIB=$PWD/gasfm_amd/$L timeout -k 10 120 python tools/attn_bench.py --points $P 2>/dev/null | grep "segment order") || exit 1
    echo "$L points $P $r"
  done
done
# result (one box): config 4 bwd 251.6 / 254.9 us strict vs 251.4 / 248.3 loose; 25k points 32.5 / 32.5 vs 32.6 / 32.5:
# the store waits are hidden by the other waves; the variant (a GASFM_GLDS_BWD_WAIT_LOOSE patch of gat_attn.hip) was not kept
