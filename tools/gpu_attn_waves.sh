# Round 6: the grouped point-direction forward by rows per iteration (GASFM_ATTN_GRP) and wave cap (GASFM_ATTN_WAVES)
mkdir -p gpurun_out
for G in 4 8 48; do for W in 0 6144 4096 3072 2048; do
  r=$(GASFM_ATTN_GRP=$G GASFM_ATTN_WAVES=$W timeout -k 10 120 python tools/attn_bench.py 2>/dev/null | grep "segment order") || exit 1
  echo "grp $G waves $W $r"
done; done
