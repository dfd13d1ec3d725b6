"""Per-kernel totals of ONE replayed step from a rocprofv3 kernel-trace database (full names).

usage: python tools/kernel_table.py <run_results.db> [step_index] [top]
"""
import re
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*$", "", n)
    n = re.sub(r"^at::native::vectorized_elementwise_kernel<4, at::native::", "vec<", n)
    return n[:80]


def main():
    db = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    st = [i for i, r in enumerate(rows) if "edge0_prologue_fwd" in r[0]]
    seg = rows[st[k]:st[k + 1]]
    d = defaultdict(lambda: [0, 0.0])
    for n, s, e in seg:
        d[short(n)][0] += 1
        d[short(n)][1] += (e - s) / 1e3
    print(f"step {k}: {len(seg)} kernels, busy {sum(v[1] for v in d.values()) / 1e3:.2f} ms")
    for name, (n, t) in sorted(d.items(), key=lambda x: -x[1][1])[:top]:
        print(f"  {t:8.1f} us {n:5d} x {t / n:7.2f}  {name}")


if __name__ == "__main__":
    main()
