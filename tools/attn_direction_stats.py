"""Edge-sized attention kernels of a rocprofv3 kernel trace, split by graph direction.

usage: python tools/attn_direction_stats.py <run_results.db> [steps_to_skip]

Every block's forward launches its two edge-sized GATv2 attentions in a fixed order -- the point
direction (proj2scenepoint, the bench's roofline kernel) first, then the camera direction
(proj2view) -- followed by the global graphs' small kernels (Geom<1024,256>, Geom<64,16>).  The
k-th edge-sized forward launch of a step is therefore the point direction for even k; the
backward (DualAttentionFn.backward) also runs the point direction first, then the camera
direction.  (Round-2 profiles before this note labelled the backward the other way round.)  Prints per
(kernel, direction): launches, mean / min / max microseconds and workgroups, over the steps
after the first ``steps_to_skip`` (default 2, the warm-up).
"""
import re
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x / workgroup_x from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if "edge0_prologue_fwd" in r[0]]
    if len(starts) <= skip:
        print("not enough steps in the trace")
        return
    stats = defaultdict(list)
    for a, b in zip(starts[skip:], starts[skip + 1:] + [len(rows)]):
        seen = defaultdict(int)
        for name, s, e, wgs in rows[a:b]:
            if not re.search(r"attn_(fwd|bwd)", name) or "combine" in name:
                continue
            if re.search(r"Geom<(1024, 256|64, 16)>", name):
                continue  # the global graphs (views -> global, points -> global)
            kern = re.sub(r"\(.*", "", name.replace("void ", "").replace("(anonymous namespace)::", "").replace("gasfm::", ""))
            kind = "bwd" if "bwd" in kern else "fwd"
            k = seen[kind]
            seen[kind] += 1
            point = k % 2 == 0
            stats[(kind, kern, "point (proj2scenepoint)" if point else "camera (proj2view)")].append(((e - s) / 1e3,
                                                                                                     wgs))
    print(f"{'pass':4s} {'kernel':44s} {'direction':24s} {'launches':>8s} {'mean_us':>8s} {'min_us':>8s} "
          f"{'max_us':>8s} {'WGs':>6s}")
    for (kind, kern, d), v in sorted(stats.items()):
        t = [x for x, _ in v]
        print(f"{kind:4s} {kern[:44]:44s} {d:24s} {len(v):8d} {sum(t) / len(t):8.1f} {min(t):8.1f} {max(t):8.1f} "
              f"{v[0][1]:6d}")


if __name__ == "__main__":
    main()
