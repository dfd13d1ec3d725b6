"""Per-kernel HBM traffic per launch from FETCH_SIZE / WRITE_SIZE counter directories (tools/pmc_kernels.sh).

usage: python tools/pmc_kernel_table.py <FETCH_SIZE dir> <WRITE_SIZE dir>
FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE counts 1/2 of the bytes of 16-B-per-lane streaming reads, so reads are doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Algorithmic bytes (config 4) are
printed beside the measured ones where known.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

ALGO_MB = {  # config 4 algorithmic bytes per launch, DESIGN.md §5
    "edge_prologue_fwd_kernel<true>": 1550, "edge_epilogue_fwd_kernel": 1110, "edge_epilogue_bwd_kernel": 1090,
    "segment_rowsum_kernel": 554, "edge_prologue_bwd_kernel<true, true>": 2560,
    "point_tail_fwd_t_kernel<true>": 128, "point_hub_fwd_t_kernel<true>": 154, "point_head_fwd_kernel": 54,
    "embed2_fwd_kernel": 64, "embed2_bwd_kernel": 64,
    # round 3: fused camera-attention + prologue backward, forward seam, point backward
    "edge_cam_pbwd_kernel<true, true>": 2049, "edge_seam_fwd_kernel<true>": 1601,
    "point_hub_bwd_r_kernel<true>": 256, "point_tail_bwd_r_kernel<true>": 205,
    "attn_bwd_glds_kernel<gasfm::Geom<32, 8> >": 1120,
    # round 3, edge epilogue backward folded into edge_cam_pbwd (+ P0 read, dP0 written: 16 B per edge)
    "edge_cam_pbwd_kernel<true, true, false, false>": 2049, "edge_cam_pbwd_kernel<true, true, true, true>": 2113,
    "edge_cam_pbwd_kernel<true, true, false, true>": 2081,
    # the seam kernel's two modes (32-wide epilogue / block 0's 2-wide one: P 8 + P' 128 + XL 128 + pt, pos 8)
    "edge_seam_fwd_kernel<true, false>": 1601, "edge_seam_fwd_kernel<true, true>": 1088,
    # round 4: the pbwd kernels carry a fifth template argument (XP: dXLp gathered through pos)
    "edge_cam_pbwd_kernel<true, true, true, true, false>": 2113,
    "edge_cam_pbwd_kernel<true, true, false, true, false>": 2081,
    # round 4: EPI became an int template argument (1: the 32-wide fold; 2: block 0's, + aux 16 B per edge)
    "edge_cam_pbwd_kernel<true, true, 1, true, false>": 2113,
    "edge_cam_pbwd_kernel<true, true, 0, true, false>": 2081,
    "edge_cam_pbwd_kernel<true, true, 2, true, false>": 2145,
}


def per_kernel(d, counter):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                k = re.sub(r"\(.*", "", row["Kernel_Name"].replace("(anonymous namespace)::", ""))
                k = k.replace("void ", "").replace("gasfm::", "")
                out[k].append(float(row["Counter_Value"]) * 1024)
    return out


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    print(f"{'kernel':45s} {'launches':>8s} {'read MB':>9s} {'write MB':>9s} {'total MB':>9s} {'algo MB':>8s} ratio")
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        rd = 2 * sum(f) / len(f) / 1e6 if f else float("nan")
        wr = sum(w) / len(w) / 1e6 if w else float("nan")
        algo = ALGO_MB.get(k)
        ratio = f"{(rd + wr) / algo:.2f}" if algo else "-"
        print(f"{k[:45]:45s} {len(f):8d} {rd:9.1f} {wr:9.1f} {rd + wr:9.1f} {algo or '-':>8} {ratio}")


if __name__ == "__main__":
    main()
