# Round 6: whole-scene camera piece length (GASFM_DEFAULT_PIECE) at config 4: per-kernel times of the camera-item
# edge kernels (rocprof stats) and the step, per setting
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for P in 256 224 192 256 224 160; do
  GASFM_DEFAULT_PIECE=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc_$P -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > /tmp/pc_$P.log 2>&1 || { tail -20 /tmp/pc_$P.log; exit 1; }
  f=$(find /tmp/pc_$P -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "piece=$P" <<'PY' | tee -a $R/gpurun_out/pc_kstats.txt
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if re.search(r"edge_seam_fwd|edge_cam_pbwd|attn_combine|attn_bwd_combine", n):
        short = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void gasfm::", "").replace("gasfm::", ""))
        out.append(f"  {short:52s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs']) / 1e3:8.2f} total_ms {float(r['TotalDurationNs']) / 1e6:8.3f}")
print("==", sys.argv[2]); print("\n".join(out))
PY
  rm -rf /tmp/pc_$P
  cd $R
  GASFM_DEFAULT_PIECE=$P timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/pc_c4.json 2> gpurun_out/pc_c4.err || { tail -20 gpurun_out/pc_c4.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/pc_c4.json').read().strip().splitlines()[-1]);print('config4 piece=$P', round(d['ms_per_step'],3))" | tee -a gpurun_out/pc_kstats.txt
  cd /tmp
done
