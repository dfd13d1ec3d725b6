"""Time ESFMLoss at config 4 (m = 1000, n = 200k, ~4M edges) on the GPU box.

usage: python tools/loss_bench.py [--reps R]
Lines (JSON): the HIP loss kernels one by one (HIP events on the launch stream) with achieved
GB/s from their algorithmic bytes, the whole HIP loss forward+backward, and the
reference formulation (code/loss_functions.py:85-123: dense Ps @ pts3D [m, 3, n], masks,
gradient hook) run by torch on the same GPU for comparison.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gasfm_amd import Conf, SceneData, _native, synthetic  # noqa: E402
from gasfm_amd.loss import ESFMLoss, _edge_tensors  # noqa: E402


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


def dense_reference_loss(Ps, pts3D, norm_M, valid, margin=1e-4, w=1.0):
    """The reference's ESFMLoss.forward for the conf/learning loss section, on dense tensors."""
    pts_2d = Ps @ pts3D
    mask = pts_2d[:, 2, :] >= margin
    npos = max(1, torch.sum(valid & mask).item())
    pts_2d.register_hook(lambda g: torch.where(mask[:, None, :].repeat(1, 3, 1), F.normalize(g, dim=1) / npos, g))
    hinge = (margin - pts_2d[:, 2, :]) * w
    pts_2d = pts_2d / torch.where(mask, pts_2d[:, 2, :], torch.ones_like(mask).float()).unsqueeze(1)
    reproj = (pts_2d[:, 0:2, :] - norm_M.reshape(Ps.shape[0], 2, -1)).norm(dim=1)
    return torch.where(mask, reproj, hinge)[valid].mean()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-dense", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = synthetic.config4()
    data = SceneData.from_synthetic(sc).to(dev)
    E, m, n = sc.num_edges, sc.m, sc.n
    g = torch.Generator(device=dev).manual_seed(0)
    Ps = torch.zeros((m, 3, 4), device=dev)
    Ps[:, :, :3] = torch.eye(3, device=dev) + 0.1 * torch.randn((m, 3, 3), device=dev, generator=g)
    Ps[:, :, 3] = 0.3 * torch.randn((m, 3), device=dev, generator=g)
    X = torch.randn((4, n), device=dev, generator=g)
    X[2] = 2.0 + 1.5 * X[2]
    X[3] = 1.0
    conf = Conf({"model": {"view_head": {"enabled": True}, "scenepoint_head": {"enabled": True}},
                 "loss": {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
                          "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True,
                          "hinge_loss_weight": 1.0}})
    lossf = ESFMLoss(conf)
    res = []

    def report(name, us, nbytes=None, **kw):
        r = {"op": name, "us": round(us, 1), **kw}
        if nbytes:
            r["GBps"] = round(nbytes / us / 1e3, 1)
        res.append(r)
        print(json.dumps(r), flush=True)

    (cam, pt), vals, cptr, pptr, perm = _edge_tensors(data)
    P = Ps.reshape(m, 12).contiguous()
    part = torch.empty((_native.esfm_part_rows(E), 2), device=dev)
    margin, w, hinge, eq, vo = lossf.kernel_conf()
    # algorithmic bytes: per edge cam + pt + 2 values (16 B) + each point's 4 coords once + cameras once
    fwd_bytes = 16 * E + 16 * n + 48 * m
    report("esfm_fwd", _time(lambda: _native.esfm_fwd(cam, pt, vals, P, X, margin, w, hinge, part), args.reps),
           fwd_bytes)
    # compute_core_errors' reprojection error (gasfm_reproj_error): same bytes as esfm_fwd
    report("reproj_error", _time(lambda: _native.reproj_error(cam, pt, vals, P, X), args.reps), fwd_bytes)
    tot = _native.colsum(part)
    dloss = torch.ones(1, device=dev)
    dP, dX = torch.empty_like(P), torch.empty_like(X)
    # camera pass: pt + 2 values per edge + point coords; point pass: perm + cam + 2 values per edge + dX
    bwd_bytes = (12 * E + 16 * n + 48 * m) + (16 * E + 32 * n + 4 * n + 48 * m)
    report("esfm_bwd (cam + pt kernels)",
           _time(lambda: _native.esfm_bwd(cptr, pptr, perm, cam, pt, vals, P, X, margin, w, hinge, eq, vo, dloss,
                                          tot, dP, dX), args.reps), bwd_bytes)

    Pr, Xr = Ps.clone().requires_grad_(True), X.clone().requires_grad_(True)

    def hip_step():
        Pr.grad = Xr.grad = None
        lossf({"Ps_norm": Pr, "pts3D": Xr}, data).backward()

    report("ESFMLoss fwd+bwd (HIP, autograd)", _time(hip_step, args.reps), E=E)
    if not args.no_dense:
        nm = torch.zeros((m, n, 2), device=dev)
        nm[data.x.indices[0], data.x.indices[1]] = data.x.values
        norm_M = nm.permute(0, 2, 1).reshape(2 * m, n)
        valid = torch.zeros((m, n), dtype=torch.bool, device=dev)
        valid[data.x.indices[0], data.x.indices[1]] = True

        def dense_step():
            Pr.grad = Xr.grad = None
            dense_reference_loss(Pr, Xr, norm_M, valid).backward()

        report("reference formulation fwd+bwd (torch dense, same GPU)", _time(dense_step, max(3, args.reps // 4)),
               E=E)


if __name__ == "__main__":
    main()
