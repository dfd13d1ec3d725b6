"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite output).

usage: python tools/rocprof_summary.py <run_results.db> <out.csv> [steps]
Writes name, calls, total_ms, avg_us, pct (the --stats columns) sorted by total time, and
prints the top 25 with per-step milliseconds when the number of profiled steps is given.
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                     "max(end - start) from kernels group by name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", r[4], r[5], f"{100.0 * r[2] / tot:.2f}"])
    print(f"total kernel time {tot / 1e6:.2f} ms" + (f" ({tot / 1e6 / steps:.2f} ms/step)" if steps else ""))
    for r in rows[:25]:
        per = f"{r[2] / 1e6 / steps:7.2f} ms/step" if steps else ""
        print(f"{r[2] / 1e6:9.2f} ms {r[1]:6d} x {r[3] / 1e3:8.1f} us {per}  {r[0][:100]}")


if __name__ == "__main__":
    main()
