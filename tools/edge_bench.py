"""Time the per-edge block kernels and the point-node kernels alone at config-4 sizes (GPU box).

usage: python tools/edge_bench.py [--reps R]
One JSON line per kernel: mean launch time (HIP events on the launch stream) and achieved
GB/s from the algorithmic bytes of DESIGN.md §5.  GASFM_LIB selects an A/B library variant.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gasfm_amd import SceneData, _native, synthetic  # noqa: E402


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=200_000, help="points (25000: the per-rank load at 8 GPUs)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = synthetic.config4() if args.n == 200_000 else synthetic.windowed_scene(1000, args.n, seed=4)
    data = SceneData.from_synthetic(sc).to(dev)
    E, m, n = sc.num_edges, sc.m, sc.n
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    P, P0, dPo = rnd(E, 32), rnd(E, 2), rnd(E, 32)
    XL, dXL = torch.empty(E, 64, device=dev), rnd(E, 64)
    ln_w, ln_b = 1 + 0.1 * rnd(32), 0.1 * rnd(32)
    W, b = rnd(64, 32) / 6, rnd(64)
    Wp, bp = rnd(32, 34) / 6, rnd(32)
    Sp, Sv, Sg = rnd(n, 32), rnd(m, 32), rnd(32)
    cam = data.x.indices[0].to(torch.int32).contiguous()
    pt = data.x.indices[1].to(torch.int32).contiguous()
    pp = data.graph_wrappers["proj2scenepoint"].plan
    pc = data.graph_wrappers["proj2view"].plan
    out, dP = torch.empty_like(P), torch.empty_like(P)
    res = []

    def run(name, fn, nbytes):
        t = _time(fn, args.reps)
        res.append({"kernel": name, "us": round(t, 1), "GBps": round(nbytes / t / 1e3, 1),
                    "lib": os.environ.get("GASFM_LIB", "default")})
        print(json.dumps(res[-1]), flush=True)

    run("edge_prologue_fwd(LN, pos)",
        lambda: _native.edge_prologue_fwd(P, ln_w, ln_b, 1e-5, W, b, XL, pp.pos), E * (128 + 256 + 4))
    run("edge_epilogue_fwd",
        lambda: _native.edge_epilogue_fwd(P, P0, cam, pt, ln_w, ln_b, 1e-5, Wp, bp, Sp, Sv, Sg, 0.25, out),
        E * 272 + (n + m) * 128)
    dSv = torch.empty(m, 32, device=dev)
    part_dsv = torch.empty(max(pc.n_part_rows, 1), 32, device=dev)
    dP0 = torch.empty(E, 2, device=dev)
    wg = _native.edge_part_floats(1, E, pc.n_items) // (32 * 34)
    part_w = torch.empty(wg, 32 * 34, device=dev)
    run("edge_epilogue_bwd",
        lambda: _native.edge_epilogue_bwd(pc.items, pc.n_items, dPo, P, P0, ln_w, ln_b, 1e-5, Wp, 0.25, dSv,
                                          part_dsv, dP0, part_w), E * 272)
    rows = _native.edge_part_floats(0, E) // (64 * 32 + 128)
    part = torch.empty(rows, 64 * 32 + 128, device=dev)
    run("edge_prologue_bwd(LN, RES)",
        lambda: _native.edge_prologue_bwd(dXL, P, dPo, ln_w, ln_b, 1e-5, W, Wp, 0.25, dP, part), E * 640)
    # prologue + camera attention (csrc/edge_cam.hip) on the camera plan, and its backward
    XLp = torch.empty(E, 32, device=dev)
    XRc, att, bias = rnd(m, 32), rnd(32) / 4, rnd(32)
    co, cmax, csum = torch.empty(m, 32, device=dev), torch.empty(m, 4, device=dev), torch.empty(m, 4, device=dev)
    cpart = torch.empty(max(pc.n_part_rows, 1), 40, device=dev)
    run("edge_cam_fwd(LN, pos)",
        lambda: _native.edge_cam_fwd(P, ln_w, ln_b, 1e-5, W[:32].contiguous(), b[:32].contiguous(),
                                     W[32:].contiguous(), b[32:].contiguous(), XLp, pp.pos, XRc, att, bias, 0.2,
                                     pc.items, pc.n_items, True, co, cmax, csum, cpart),
        E * (128 + 128 + 4) + m * 128)
    Pn = torch.empty_like(P)
    run("edge_seam_fwd(epilogue + cam)",
        lambda: _native.edge_seam_fwd(P, P0, pt, ln_w, ln_b, 1e-5, Wp, bp, Sp, Sv, Sg, 0.25, Pn, ln_w, ln_b, 1e-5,
                                      W[:32].contiguous(), b[:32].contiguous(), W[32:].contiguous(),
                                      b[32:].contiguous(), XLp, pp.pos, XRc, att, bias, 0.2, pc.items, pc.n_items,
                                      True, co, cmax, csum, cpart),
        E * (128 + 8 + 4 + 128 + 128 + 128 + 4) + (n + m) * 128)
    dXLc, dXRc = torch.empty(E, 32, device=dev), torch.empty(m, 32, device=dev)
    pdxr = torch.empty(max(pc.n_part_rows, 1), 32, device=dev)
    r_, c_ = _native.edge_cam_bwd_part_shape(pc.n_items)
    cbp = torch.empty(r_, c_, device=dev)
    gout = rnd(m, 32)
    run("edge_cam_bwd(LN)",
        lambda: _native.edge_cam_bwd(P, ln_w, ln_b, 1e-5, W[32:].contiguous(), b[32:].contiguous(), XRc, att, bias,
                                     0.2, co, cmax, csum, gout, pc.items, pc.n_items, dXLc, dXRc, pdxr, cbp),
        E * (128 + 128) + m * 256)
    dXLp_in, dRes_in = rnd(E, 32), rnd(E, 32)
    rp, cp_ = _native.edge_cam_pbwd_part_shape(pc.n_items)
    pbp = torch.empty(rp, cp_, device=dev)
    run("edge_cam_pbwd(LN, RES)",
        lambda: _native.edge_cam_pbwd(P, ln_w, ln_b, 1e-5, W[:32].contiguous(), W[32:].contiguous(),
                                      b[32:].contiguous(), Wp, 0.25, XRc, att, bias, 0.2, co, cmax, csum, gout,
                                      pc.items, pc.n_items, dXLp_in, dRes_in, dP, dXRc, pdxr, pbp),
        E * 512 + m * 256)
    # with the edge epilogue's backward folded in (edge_block.EPI_FOLD): EPI, DWP, both
    P0f, dP0f, dSvf = rnd(E, 2), torch.empty(E, 2, device=dev), torch.empty(m, 32, device=dev)
    pdsv = torch.empty(max(pc.n_part_rows, 1), 32, device=dev)
    rpw, cpw = _native.edge_cam_pbwd_part_shape(pc.n_items, 34)
    pbw = torch.empty(rpw, cpw, device=dev)
    for tag, epi, dwp in (("EPI", True, False), ("DWP", False, True), ("EPI+DWP", True, True)):
        run(f"edge_cam_pbwd(LN, RES, {tag})",
            lambda epi=epi, dwp=dwp: _native.edge_cam_pbwd(
                P, ln_w, ln_b, 1e-5, W[:32].contiguous(), W[32:].contiguous(), b[32:].contiguous(), Wp, 0.25, XRc,
                att, bias, 0.2, co, cmax, csum, gout, pc.items, pc.n_items, dXLp_in, dRes_in, dP, dXRc, pdxr, pbw,
                epi=(Wp, 0.25, dSvf, pdsv, dP0f) if epi else None, dwp=P0f if dwp else None),
            E * 528 + m * 256)
    dSp = torch.empty(n, 32, device=dev)
    run("segment_rowsum", lambda: _native.segment_rowsum(pp.items, pp.n_items, pp.perm, dPo, 0.25, dSp, None),
        E * 132 + n * 128)
    # point-node kernels (n x 64)
    X = rnd(n, 64)
    g64, b64 = 1 + 0.1 * rnd(64), 0.1 * rnd(64)
    for n_out, resid in ((32, False), (64, True)):
        Wn, bn = rnd(n_out, 64) / 8, rnd(n_out)
        Y = torch.empty(n, n_out, device=dev)
        dY = rnd(n, n_out)
        dX = torch.empty_like(X)
        nrows = _native.node_part_rows(n, n_out, resid)
        npart = torch.empty(nrows, n_out * 64 + n_out + 128, device=dev)
        run(f"node_fwd<{n_out},{int(resid)}>",
            lambda: _native.node_ln_linear_fwd(X, g64, b64, 1e-5, Wn, bn, resid, Y), n * (256 + 4 * n_out))
        run(f"node_bwd<{n_out},{int(resid)}>",
            lambda: _native.node_ln_linear_bwd(dY, X, g64, b64, 1e-5, Wn, resid, dX, npart),
            n * (4 * n_out + 512))
    point_bench(run, rnd, n, dev)


def point_bench(run, rnd, n, dev):
    """Fused scene-point tail / hub kernels (csrc/point_block.hip) at n rows."""
    from gasfm_amd import point_block as pb
    X, agg = rnd(n, 64), rnd(n, 32)
    g64, b64 = 1 + 0.1 * rnd(64), 0.1 * rnd(64)
    Wp, bp, Wm, bm = rnd(64, 32) / 6, rnd(64), rnd(64, 64) / 8, rnd(64)
    out = torch.empty(n, 64, device=dev)
    run("point_tail_fwd", lambda: _native.point_tail_fwd(X, agg, Wp, bp, g64, b64, 1e-5, Wm, bm, out), n * 640)
    dx, dagg = torch.empty(n, 64, device=dev), torch.empty(n, 32, device=dev)
    rows, cols = _native.point_tail_part_shape(n, True)
    part = torch.empty(rows, cols, device=dev)
    dout = rnd(n, 64)
    run("point_tail_bwd", lambda: _native.point_tail_bwd(dout, X, agg, Wp, bp, g64, b64, 1e-5, Wm, dx, dagg, part),
        n * 1152)
    WA, WB, bB, WC, bWC, WD, bD = rnd(32, 64) / 8, rnd(64, 64) / 8, rnd(64), rnd(32, 64) / 8, rnd(32), rnd(32, 32) / 6, rnd(32)
    SA, XL, XR = torch.empty(n, 32, device=dev), torch.empty(n, 64, device=dev), torch.empty(n, 32, device=dev)
    run("point_hub_fwd", lambda: _native.point_hub_fwd(X, 1e-5, g64, b64, WA, SA, WB, bB, XL, g64, b64, WC, bWC, WD,
                                                        bD, XR), n * 768)
    dSA, dXL, dXR, dsk = rnd(n, 32), rnd(n, 64), rnd(n, 32), rnd(n, 64)
    rc, cc = _native.point_hub_part_shape(n, 1, True)
    ra, ca = _native.point_hub_part_shape(n, 0, True)
    pc_, pa_ = torch.empty(rc, cc, device=dev), torch.empty(ra, ca, device=dev)
    dp = torch.empty(n, 64, device=dev)
    run("point_hub_bwd_c", lambda: _native.point_hub_bwd_c(X, 1e-5, g64, b64, WC, bWC, WD, dXR, dsk, dp, pc_),
        n * 640)
    run("point_hub_bwd_ab", lambda: _native.point_hub_bwd_ab(X, 1e-5, g64, b64, WA, WB, dSA, dXL, dp, dp, pa_),
        n * 1024)
    del pb


if __name__ == "__main__":
    main()
