# Round 6: the fused point tail + hub forward at 4- vs 6-wave workgroups (GASFM_TAIL_HUB_WAVES): parity,
# per-kernel times (proxy, config 4), proxy steps alternating
# (the GASFM_TAIL_HUB_WAVES knob was removed after this A/B: 4-wave workgroups kept, profiles/r6_ab_tail_hub.txt)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_point_block.py -k fused > gpurun_out/thw_tests.log 2>&1 || { tail -30 gpurun_out/thw_tests.log; exit 1; }
tail -1 gpurun_out/thw_tests.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for NW in 6 4; do
  for W in 8 1; do
    GASFM_TAIL_HUB_WAVES=$NW timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/thw_${NW}_$W -o run -- python3 $R/bench.py --emulate-world $W --steps 5 --warmup 2 --no-cpu-baseline > /tmp/thw_${NW}_$W.log 2>&1 || { tail -20 /tmp/thw_${NW}_$W.log; exit 1; }
    f=$(find /tmp/thw_${NW}_$W -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "waves=$NW emulate_world=$W" <<'PY' | tee -a $R/gpurun_out/thw_kstats.txt
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
cd $R
for NW in 6 4 6 4; do
  GASFM_TAIL_HUB_WAVES=$NW timeout -k 10 200 python bench.py --emulate-world 8 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/thw_em8.json 2> gpurun_out/thw_em8.err || { tail -20 gpurun_out/thw_em8.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/thw_em8.json').read().strip().splitlines()[-1]);print('em8 waves=$NW', round(d['ms_per_step'],3))"
done
