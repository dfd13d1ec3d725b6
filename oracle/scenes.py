"""Scene -> oracle Graph, restated in numpy — TEST INFRASTRUCTURE (oracle).

Follows the reference's graph build independently of gasfm_amd:
  get_M_valid_points  utils/dataset_utils.py:86-113 ((x,y) != (0,0), >= 2 views per point)
  M2sparse            utils/dataset_utils.py:116-156 (np.nonzero row-major -> cam-major edges,
                      values = (N [x y 1]^T)[:2], geo_utils.normalize_M 689-703)
  valid views/points  datasets/SceneData.py:174-187 (>= 8 points per view, >= 2 views per point)
"""
import numpy as np
import torch

from .gasfm_ref import Graph


def graph_from_dense(M, Ns, fp32_values=False):
    """M [2m, n] pixels (0 = unobserved), Ns [m, 3, 3] -> (values [E, 2] float64, Graph).

    fp32_values: normalise as the reference does on its float32 M / Ns (geo_utils.normalize_M,
    geo_utils.py:689-703: a batched fp32 ``Ns @ [x; y; 1]``), then widen to float64."""
    M = np.asarray(M, dtype=np.float64)
    Ns = np.asarray(Ns, dtype=np.float64)
    m, n = M.shape[0] // 2, M.shape[1]
    M3 = M.reshape(m, 2, n).swapaxes(1, 2)                # (m, n, 2)
    valid = np.abs(M3).sum(axis=2) != 0
    valid[:, valid.sum(axis=0) < 2] = False
    cam, pt = np.nonzero(valid)                          # row-major == cam-major
    h = np.concatenate([M3, np.ones((m, n, 1))], axis=2)  # (m, n, 3)
    if fp32_values:
        M32 = torch.from_numpy(np.asarray(M, dtype=np.float32)).reshape(m, 2, n)
        h32 = torch.cat([M32, torch.ones((m, 1, n), dtype=torch.float32)], 1)
        norm32 = (torch.from_numpy(Ns.astype(np.float32)) @ h32).permute(0, 2, 1)[:, :, :2]
        values = norm32.numpy()[cam, pt].astype(np.float64)
    else:
        norm = np.einsum("mij,mnj->mni", Ns, h)[:, :, :2]
        values = norm[cam, pt]
    return values, graph_from_edges(cam, pt, m, n)


def graph_from_edges(cam, pt, m, n):
    cam = np.asarray(cam, dtype=np.int64)
    pt = np.asarray(pt, dtype=np.int64)
    pts_per_cam = np.bincount(cam, minlength=m)
    cams_per_pt = np.bincount(pt, minlength=n)
    return Graph(cam=torch.from_numpy(cam), pt=torch.from_numpy(pt), m=m, n=n,
                 valid_views=torch.from_numpy(np.nonzero(pts_per_cam >= 8)[0]),
                 valid_pts=torch.from_numpy(np.nonzero(cams_per_pt >= 2)[0]))
