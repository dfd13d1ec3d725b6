"""Per-kernel-name totals of ONE step from a rocprofv3 kernel-trace database (full template names).

usage: python tools/step_kernels.py <run_results.db> [step_index] [regex]
Steps are delimited by the block-0 prologue kernel, as tools/step_breakdown.py.
"""
import re
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    st = [i for i, r in enumerate(rows) if "edge0_prologue_fwd" in r[0]]
    tot, cnt = defaultdict(float), defaultdict(int)
    for n, s, e in rows[st[k]:st[k + 1]]:
        n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
        if pat is None or pat.search(n):
            tot[n] += (e - s) * 1e-3
            cnt[n] += 1
    for n in sorted(tot, key=lambda x: -tot[x]):
        print(f"{tot[n]:9.1f} us {cnt[n]:5d} x {tot[n] / cnt[n]:7.1f} us  {n[:110]}")


if __name__ == "__main__":
    main()
