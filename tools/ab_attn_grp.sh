# A/B of the attention forward variants (GASFM_ATTN_GRP) on the config-4 plans: one process each
set -e
for v in "$@"; do
  echo "GASFM_ATTN_GRP=$v"
  GASFM_ATTN_GRP=$v timeout -k 10 200 python tools/attn_layout_probe.py --reps 7 | grep contiguous
done
