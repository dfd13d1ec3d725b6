set -e
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/prof_ts -o run -- python3 $ROOT/tools/host_profile.py --steps 2 --top 5 > $ROOT/gpurun_out/ts.log 2>&1
cd $ROOT && python - <<'PY'
import sqlite3
c = sqlite3.connect("gpurun_out/prof_ts/run_results.db")
rows = c.execute("select name, start, end from kernels order by start").fetchall()
t0, t1 = rows[0][1], rows[-1][2]
busy = sum(e - s for _, s, e in rows)
print("kernels", len(rows), "span ms", (t1 - t0) / 1e6, "busy ms", busy / 1e6)
PY
grep "per step" gpurun_out/ts.log
