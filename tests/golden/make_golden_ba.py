"""Generate tests/golden/ba.npz from the REFERENCE's own geometry helpers (build container only).

    python tests/golden/make_golden_ba.py

The bundle adjustment itself runs in Ceres (absent offline), but everything around it in
ba_functions.euc_ba (utils/ba_functions.py:6-72) is numpy in utils/geo_utils.py, imported in
place here (tests/golden/refimport.py): camera matrices (batch_get_camera_matrix_from_rtk,
:307-315), reprojection errors (reprojection_error_with_points, :371-391), the normalisation
(normalize_points_cams, :536-560) and the DLT triangulation (dlt_triangulation, :611-656).
They run on a synthetic BA scene (gasfm_amd.synthetic.ba_scene: 12 cameras, 150 points, 4..7
views, 0.5 px noise, perturbed cameras) and the outputs pin oracle/ba.py's restatements.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refimport  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402  (input generation only)


def main():
    refimport.load()
    import importlib
    geo = importlib.import_module("utils.geo_utils")
    sc = synthetic.ba_scene(12, 150, 5, noise_px=0.5, seed=7)
    xs, Rs, ts, Ks = sc["xs"], sc["Rs"], sc["ts"], sc["Ks"]
    rng = np.random.default_rng(8)
    # drop a few observations so view counts are ragged (2..5), one point left with a single view
    drop = rng.random(xs.shape[:2]) < 0.15
    xs[drop] = 0
    seen0 = np.nonzero(np.abs(xs[:, 0]).sum(1) != 0)[0]
    xs[seen0[1:], 0] = 0  # point 0: a single view (filtered out, NaN in the triangulation)
    ts_p = ts + 0.02 * rng.standard_normal(ts.shape)
    Ps = geo.batch_get_camera_matrix_from_rtk(Rs, ts_p, Ks)
    Ns = np.linalg.inv(Ks)
    vis = geo.xs_valid_points(xs)
    vis = vis.numpy() if hasattr(vis, "numpy") else np.asarray(vis)
    nP, nx = geo.normalize_points_cams(Ps, xs, Ns)
    X = geo.dlt_triangulation(nP, nx, vis)
    err = geo.reprojection_error_with_points(Ps, X, xs, vis)
    Xp = np.concatenate([sc["Xs"], np.ones((150, 1))], axis=1)
    err_gt = geo.reprojection_error_with_points(Ps, Xp, xs, vis)
    out = dict(xs=xs, Rs=Rs, ts=ts_p, Ks=Ks, Ps=Ps, vis=vis, norm_P=nP, norm_x=nx, X_dlt=X, err_dlt=err,
               X_gt=sc["Xs"], err_gt=err_gt)
    path = os.path.join(HERE, "ba.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, "visible", int(vis.sum()), "nan points", int(np.isnan(X[:, 0]).sum()))


if __name__ == "__main__":
    main()
