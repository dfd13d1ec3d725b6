"""Kernel-time breakdown of ONE replayed step from a rocprofv3 kernel-trace database.

usage: python tools/step_breakdown.py <run_results.db> [step_index]
Steps are delimited by the block-0 prologue kernel (first kernel of every forward).
"""
import re
import sqlite3
import sys
from collections import defaultdict

CATS = [
    ("edge kernels", r"edge_|edge0_|segment_rowsum"),
    ("attention", r"attn_"),
    ("node kernels", r"node_(fwd|bwd)"),
    ("global vec", r"gvec_"),
    ("colsum", r"colsum"),
    ("hipBLASLt GEMM", r"^Cijk_"),
    ("torch LayerNorm", r"layer_norm|GammaBeta|GradInput|cuComputePartGrad|cuComputeGrad"),
    ("torch reduce", r"reduce_kernel"),
    ("torch add", r"CUDAFunctor_add"),
    ("torch fill/copy/cat", r"Fill|copyBuffer|fillBuffer|CatArray|direct_copy|copy_kernel"),
    ("torch relu/threshold/mul", r"clamp|threshold|BinaryFunctor|MulFunctor|elementwise_kernel_manual"),
]


def main():
    db = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x / workgroup_x from kernels order by start").fetchall()
    st = [i for i, r in enumerate(rows) if "edge0_prologue_fwd" in r[0]]
    seg = rows[st[k]:st[k + 1]]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for n, s, e, _ in seg:
        for cat, pat in CATS:
            if re.search(pat, n):
                break
        else:
            cat = "other: " + re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))[:50]
        tot[cat] += (e - s) / 1e3
        cnt[cat] += 1
    span = (seg[-1][2] - seg[0][1]) / 1e3
    print(f"step {k}: {len(seg)} kernels, span {span / 1e3:.2f} ms, busy {sum(tot.values()) / 1e3:.2f} ms")
    for cat in sorted(tot, key=lambda x: -tot[x]):
        print(f"  {tot[cat] / 1e3:7.2f} ms {cnt[cat]:5d} kernels  {cat}")
    per = defaultdict(lambda: [0.0, 0, 0])
    for n, s, e, wg in seg:
        key = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))[:90]
        per[key][0] += (e - s) / 1e3
        per[key][1] += 1
        per[key][2] += wg
    print("top kernels (us total, count, us mean, mean workgroups):")
    for key in sorted(per, key=lambda x: -per[x][0])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
        t, n, w = per[key]
        print(f"  {t:9.1f} {n:5d} {t / n:8.2f} {w // n:7d}  {key}")


if __name__ == "__main__":
    main()
