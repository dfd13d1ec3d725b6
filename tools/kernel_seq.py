"""Kernel sequence of one block of a replayed step (rocprofv3 kernel-trace db): duration, gap
to the previous kernel's end, workgroups, name.

usage: python tools/kernel_seq.py <run_results.db> [block] [step]
The forward of block b starts at its prologue (edge_prologue_fwd<true>, edge_cam_fwd<true> or the
forward seam edge_seam_fwd); the listing runs to the next one
(pass block -1 for the whole backward of the step instead)."""
import re
import sqlite3
import sys


def short(n):
    return re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))[:80]


def main():
    db = sys.argv[1]
    blk = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    step = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    rows = sqlite3.connect(db).execute(
        "select name, start, end, grid_x / workgroup_x from kernels order by start").fetchall()
    st = [i for i, r in enumerate(rows) if "edge0_prologue_fwd" in r[0]]
    seg = rows[st[step]:st[step + 1]]
    if blk >= 0:
        idx = [i for i, r in enumerate(seg) if "edge_prologue_fwd_kernel<true>" in r[0] or "edge_cam_fwd_kernel<true>" in r[0]
               or "edge_seam_fwd_kernel" in r[0]]
        seg = seg[idx[blk]:idx[blk + 1]]
    else:
        first_bwd = next(i for i, r in enumerate(seg) if "bwd" in r[0])
        seg = seg[first_bwd:]
    prev = None
    tot = 0.0
    for n, s, e, g in seg:
        gap = (s - prev) / 1e3 if prev else 0.0
        prev = e
        tot += (e - s) / 1e3
        print(f"{(e - s) / 1e3:7.1f} gap{gap:5.1f} {g:6d} {short(n)}")
    print(f"{len(seg)} kernels, busy {tot:.1f} us, span {(seg[-1][2] - seg[0][1]) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
