# Round 6: per-kernel times of the point tail / hub forward, fused vs two kernels (proxy and config 4)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for F in 1 0; do
  for W in 8 1; do
    GASFM_TAIL_HUB=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/thp_${F}_$W -o run -- python3 $R/bench.py --emulate-world $W --steps 5 --warmup 2 --no-cpu-baseline > /tmp/thp_${F}_$W.log 2>&1 || { tail -20 /tmp/thp_${F}_$W.log; exit 1; }
    f=$(find /tmp/thp_${F}_$W -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "tail_hub=$F emulate_world=$W" <<'PY' | tee -a $R/gpurun_out/th_kstats.txt
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("==", sys.argv[2])
for r in rows:
    n = r["Name"]
    if re.search(r"point_(tail|hub|tail_hub)_fwd", n):
        short = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void gasfm::", ""))
        print(f"  {short:42s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs']) / 1e3:8.2f} total_ms {float(r['TotalDurationNs']) / 1e6:8.3f}")
PY
  done
done
