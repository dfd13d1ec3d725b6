"""Edge-sized attention kernels of a rocprofv3 kernel trace, split by graph direction.

usage: python tools/attn_direction_stats.py <run_results.db> [steps_to_skip]

Launches are labelled by the block structure of the kernel sequence, not by a global parity:
  * blocks whose prologue is edge_cam_fwd (csrc/edge_cam.hip) run the camera direction inside
    that fused kernel, so their one edge-sized attention forward is the point direction; the
    same holds in the backward, where edge_cam_bwd follows the point-direction backward;
  * a block with a separate prologue (block 0: edge0_prologue_fwd, or edge_prologue_fwd when
    GASFM_EDGE_CAM=0) launches DualAttentionFn's two attentions point first, then camera, in
    both passes.
The global graphs' small kernels (Geom<1024,256>, Geom<64,16>) are skipped.  Prints per
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
    edge_sized = lambda n: (re.search(r"attn_(fwd|bwd)", n) and "combine" not in n
                            and not re.search(r"Geom<(1024, 256|64, 16)>", n))
    for a, b in zip(starts[skip:], starts[skip + 1:] + [len(rows)]):
        seg = rows[a:b]
        fused_fwd = False  # current forward block's prologue is edge_cam_fwd
        k_fwd = 0          # edge-sized forward launches since the block's prologue
        k_bwd = 0          # unfused backward launches since the last backward edge kernel
        for i, (name, s, e, wgs) in enumerate(seg):
            if re.search(r"edge_cam_fwd|edge_prologue_fwd|edge0_prologue_fwd", name):
                fused_fwd, k_fwd = "edge_cam_fwd" in name, 0
                continue
            if re.search(r"edge_cam_bwd|edge_prologue_bwd|edge0_prologue_bwd|edge_epilogue_bwd|edge0_epilogue_bwd",
                         name):
                k_bwd = 0
                continue
            if not edge_sized(name):
                continue
            kern = re.sub(r"\(.*", "", name.replace("void ", "").replace("(anonymous namespace)::", "").replace("gasfm::", ""))
            if "bwd" in kern:
                nxt = [r[0] for r in seg[i + 1:i + 4]]
                point = any("edge_cam_bwd" in n for n in nxt) or k_bwd % 2 == 0
                k_bwd += 1
                kind = "bwd"
            else:
                point = fused_fwd or k_fwd % 2 == 0
                k_fwd += 1
                kind = "fwd"
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
