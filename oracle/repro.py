"""Dense CPU restatement of compute_core_errors' "our_repro" -- TEST INFRASTRUCTURE (oracle).

Follows code/evaluation.py:8-31 and geo_utils.reprojection_error_with_points (geo_utils.py:371-391):
  Ps     = Ns^-1 @ Ps_norm                                  evaluation.py:22,27
  X4     = pflat(pts3D)                                     :28, geo_utils.py:332-333
  proj   = Ps @ X4  -> [m, 3, n]; visible entries / z       geo_utils.py:385-388
  errors = || xs - proj_xy ||, NaN where not visible        :389-390
  our_repro = nanmean(errors)                               evaluation.py:30
with xs = M as [m, n, 2] and visible = get_M_valid_points (>= 2 views per point).  numpy, any
float dtype.  Pinned against tests/golden/core_errors.npz, which the reference's own
compute_core_errors produced (tests/golden/make_golden_repro.py).
"""
import numpy as np


def valid_points(M):
    m = M.shape[0] // 2
    xs = M.reshape(m, 2, -1).transpose(0, 2, 1)
    v = np.abs(xs).sum(axis=2) != 0
    v[:, v.sum(axis=0) < 2] = False
    return v


def reprojection_errors(M, Ns, Ps_norm, pts3D):
    """errors [m, n] (NaN where not visible) and their nanmean."""
    m = M.shape[0] // 2
    xs = M.reshape(m, 2, -1).transpose(0, 2, 1)
    Ps = np.linalg.inv(Ns) @ Ps_norm
    vis = valid_points(M)
    with np.errstate(divide="ignore", invalid="ignore"):
        X4 = pts3D / pts3D[-1:, :]
        proj = (Ps @ X4).transpose(0, 2, 1)  # [m, n, 3]
        proj[vis] = proj[vis] / proj[vis][:, 2:3]
        err = np.linalg.norm(xs - proj[:, :, :2], axis=2)
        err[~vis] = np.nan
        return err, np.nanmean(err)
