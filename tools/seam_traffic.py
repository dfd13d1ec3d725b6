"""Launch the forward seam (edge_seam_fwd, blocks 1-11's form) alone at config 4, for counter passes
that attribute its memory traffic (round 6).  GPU box.

usage: python tools/seam_traffic.py --variant {base,sp_local,xl_seq,both} [--reps R]
  base      the model's access pattern: Sp[pt] gathered per edge in camera order (Sp is 200k x 128 B =
            25.6 MB), XL's point half scattered to pos[e] (point-segment order)
  sp_local  pt replaced by pt % 4096: the same gathers over a 512 KB table that stays in every XCD's L2
  xl_seq    pos replaced by the identity: XL rows written in edge order (streamed)
  both      the two together
Run under rocprofv3 --pmc (tools/gpu_seam_traffic.sh); every variant does the same arithmetic and
moves the same algorithmic bytes, so the counter differences are the access patterns' own cost.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gasfm_amd import SceneData, _native, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", choices=("base", "sp_local", "xl_seq", "both"), default="base")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = synthetic.config4()
    data = SceneData.from_synthetic(sc).to(dev)
    E, m, n = sc.num_edges, sc.m, sc.n
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    P, P0 = rnd(E, 32), rnd(E, 2)
    ln_w, ln_b = 1 + 0.1 * rnd(32), 0.1 * rnd(32)
    W, b = rnd(64, 32) / 6, rnd(64)
    Wp, bp = rnd(32, 34) / 6, rnd(32)
    Sp, Sv, Sg = rnd(n, 32), rnd(m, 32), rnd(32)
    pt = data.x.indices[1].to(torch.int32).contiguous()
    pp = data.graph_wrappers["proj2scenepoint"].plan
    pc = data.graph_wrappers["proj2view"].plan
    pos = pp.pos
    if args.variant in ("sp_local", "both"):
        pt = (pt % 4096).contiguous()
    if args.variant in ("xl_seq", "both"):
        pos = torch.arange(E, dtype=torch.int32, device=dev)
    XLp = torch.empty(E, 32, device=dev)
    XRc, att, bias = rnd(m, 32), rnd(32) / 4, rnd(32)
    co, cmax, csum = torch.empty(m, 32, device=dev), torch.empty(m, 4, device=dev), torch.empty(m, 4, device=dev)
    cpart = torch.empty(max(pc.n_part_rows, 1), 40, device=dev)
    Pn = torch.empty_like(P)
    Wpt, bpt, Wc, bc = W[:32].contiguous(), b[:32].contiguous(), W[32:].contiguous(), b[32:].contiguous()
    for _ in range(args.reps):
        _native.edge_seam_fwd(P, P0, pt, ln_w, ln_b, 1e-5, Wp, bp, Sp, Sv, Sg, 0.25, Pn, ln_w, ln_b, 1e-5, Wpt, bpt,
                              Wc, bc, XLp, pos, XRc, att, bias, 0.2, pc.items, pc.n_items, True, co, cmax, csum, cpart)
    torch.cuda.synchronize()
    print(f"seam {args.variant}: {args.reps} launches, E={E}", flush=True)


if __name__ == "__main__":
    main()
