"""Device bundle adjustment at scale: one euc_ba LM solve on a synthetic scene.

usage: python tools/ba_bench.py [--m 1000] [--n 200000] [--views 20] [--iters 10]

Scene: gasfm_amd.synthetic.ba_scene (cameras on a circle, windowed visibility, 0.5 px noise),
perturbed cameras and points.  Reports the problem size (edges, camera-pair blocks, edge pairs of
the reduced camera system), the setup time (pair lists, sorted once) and the mean time per LM
iteration split by pass (eval + normals, Schur build, Cholesky + solve, back-substitution + model
+ candidate cost), with cuda events around each.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import ba as B  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1000)
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--views", type=int, default=20)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--linalg", choices=("default", "magma", "cusolver"), default="default",
                    help="torch.backends.cuda.preferred_linalg_library for the Cholesky of S")
    a = ap.parse_args()
    if a.linalg != "default":
        torch.backends.cuda.preferred_linalg_library(a.linalg)
    dev = torch.device("cuda", 0)
    sc = synthetic.ba_scene(a.m, a.n, a.views, noise_px=0.5, seed=1)
    rng = np.random.default_rng(2)
    xs = torch.from_numpy(sc["xs"]).to(dev)
    Rs = torch.from_numpy(sc["Rs"]).to(dev)
    ts = torch.from_numpy(sc["ts"] + 0.01 * rng.standard_normal(sc["ts"].shape)).to(dev)
    Ks = torch.from_numpy(sc["Ks"]).to(dev)
    Xs = torch.from_numpy(sc["Xs"] + 0.01 * rng.standard_normal(sc["Xs"].shape)).to(dev)
    ed = B._Edges(xs)
    cam0, K = B._euc_params(Rs, ts, Ks)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prob = B.BAProblem("euc", cam0, Xs, ed.cidx, ed.pidx, ed.obs, K)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    f = dict(dtype=torch.float64, device=dev)
    dcam, dX = torch.zeros((a.m, 6), **f), torch.zeros((a.n, 3), **f)
    prob.evaluate(dcam, dX, True)
    prob.normals()
    prob.sc = (1.0 / (1.0 + torch.sqrt(torch.diagonal(prob.U, dim1=1, dim2=2)))).contiguous()
    prob.sp = (1.0 / (1.0 + torch.sqrt(torch.diagonal(prob.V, dim1=1, dim2=2)))).contiguous()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    tm = {"eval_normals": 0.0, "schur": 0.0, "cholesky_solve": 0.0, "backsub_model_cand": 0.0}
    L = torch.linalg
    for it in range(a.iters + 1):
        e = [ev() for _ in range(5)]
        e[0].record()
        prob.evaluate(dcam, dX, True)
        prob.normals()
        e[1].record()
        from gasfm_amd import _native
        lib = _native.lib()
        st = _native._stream(prob.obs)
        prob.bad.zero_()
        lib.gasfm_ba_damp(6, prob.m, prob.n, B._p(prob.U), B._p(prob.V), 1e3, B._p(prob.Ud), B._p(prob.Vinv),
                          B._p(prob.bad), st)
        lib.gasfm_ba_schur(6, prob.m, B._p(prob.cam_ptr), B._p(prob.cidx), B._p(prob.pidx), prob.E, B._p(prob.Jc),
                           B._p(prob.Jp), B._p(prob.Vinv), B._p(prob.gc), B._p(prob.gp), B._p(prob.Ud),
                           B._p(prob.blk_ptr), B._p(prob.blk_ab), prob.nblk, B._p(prob.pe1), B._p(prob.pe2),
                           B._p(prob.Y), B._p(prob.S), B._p(prob.rhs), st)
        e[2].record()
        Lc, info = L.cholesky_ex(prob.S)
        dc = torch.cholesky_solve(prob.rhs[:, None], Lc)[:, 0].reshape(prob.m, 6).contiguous()
        e[3].record()
        lib.gasfm_ba_backsub(6, prob.n, B._p(prob.pt_ptr), B._p(prob.perm), B._p(prob.cidx), B._p(prob.Jc),
                             B._p(prob.Jp), B._p(prob.Vinv), B._p(prob.gp), B._p(dc), B._p(prob.dp), st)
        prob.model_change(dc, prob.dp)
        prob.evaluate(dcam + dc * prob.sc, dX + prob.dp * prob.sp, False)
        e[4].record()
        torch.cuda.synchronize()
        if it:
            for k, (i, j) in zip(tm, ((0, 1), (1, 2), (2, 3), (3, 4))):
                tm[k] += e[i].elapsed_time(e[j]) / a.iters
    print(json.dumps({"scene": {"m": a.m, "n": a.n, "views": a.views, "edges": prob.E, "camera_pair_blocks": prob.nblk,
                                "edge_pairs": prob.n_pairs, "reduced_system": 6 * a.m},
                      "linalg": a.linalg, "setup_s": setup, "ms_per_lm_iteration": sum(tm.values()),
                      "ms_by_pass": tm, "info": int(info.item())}))


if __name__ == "__main__":
    main()
