# Round 6: the forward seam's traffic by access pattern (tools/seam_traffic.py): exact EA-level read /
# write bytes from separate counter passes, plus a kernel trace, per variant
set -e
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/seamtr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in base sp_local xl_seq both; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum \
    --kernel-include-regex edge_seam --output-format csv -d $OUT/${V}_rd -o run -- \
    python3 $ROOT/tools/seam_traffic.py --variant $V > $OUT/${V}_rd.txt 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    --kernel-include-regex edge_seam --output-format csv -d $OUT/${V}_wr -o run -- \
    python3 $ROOT/tools/seam_traffic.py --variant $V > $OUT/${V}_wr.txt 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/${V}_tr -o run -- \
    python3 $ROOT/tools/seam_traffic.py --variant $V > $OUT/${V}_tr.txt 2>&1
  echo "variant $V done"
done
cd $ROOT && python tools/seam_traffic_table.py $OUT base sp_local xl_seq both | tee gpurun_out/seam_traffic_table.txt
