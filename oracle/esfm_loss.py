"""Dense CPU restatement of ESFMLoss — TEST INFRASTRUCTURE (oracle).

Follows code/loss_functions.py:85-123 step by step on the dense [m, 3, n] projections:
  pts_2d = Ps @ pts3D                                   loss_functions.py:90
  mask   = z >= margin  (hinge) | |z| >= margin         :93-98, geo_utils.py:721-726
  hook on pts_2d's gradient                             :101-110
  hinge  = (margin - z) * w                             :114
  reproj = || pts_2d[:2] / where(mask, z, 1) - norm_M ||   :118-119
  loss   = where(mask, reproj, hinge)[valid].mean()     :123
and builds the dense norm_M / valid mask from the sparse edges the way SceneData does
(dataset_utils.M2sparse keeps exactly the valid entries of norm_M).  Any float dtype; autograd
through the hook gives the reference's gradients.  Pinned against tests/golden/esfm_loss.npz,
which the reference's own ESFMLoss produced (tests/golden/make_golden_loss.py).
"""
import torch
import torch.nn.functional as F


def dense_measurements(cam, pt, values, m, n, dtype=torch.float64):
    """(norm_M [2m, n], valid [m, n]) from the edge list, in the reference's layouts."""
    cam, pt = torch.as_tensor(cam, dtype=torch.int64), torch.as_tensor(pt, dtype=torch.int64)
    nm = torch.zeros((m, n, 2), dtype=dtype)
    nm[cam, pt] = torch.as_tensor(values).to(dtype)
    valid = torch.zeros((m, n), dtype=torch.bool)
    valid[cam, pt] = True
    return nm.permute(0, 2, 1).reshape(2 * m, n), valid


def esfm_loss(Ps, pts3D, norm_M, valid, margin, hinge, hinge_w, equalize, valid_only):
    m = Ps.shape[0]
    w = hinge_w if hinge else 0.0
    pts_2d = Ps @ pts3D
    z = pts_2d[:, 2, :]
    mask = (z >= margin) if hinge else (z.abs() >= margin)
    if equalize and pts_2d.requires_grad:
        if valid_only:
            npos = max(1, int(torch.sum(valid & mask).item()))
            pts_2d.register_hook(lambda g: torch.where(mask[:, None, :].repeat(1, 3, 1), F.normalize(g, dim=1) / npos,
                                                       g))
        else:
            nvalid = int(valid.sum().item())
            pts_2d.register_hook(lambda g: F.normalize(g, dim=1) / nvalid)
    hinge_term = (margin - pts_2d[:, 2, :]) * w
    div = torch.where(mask, pts_2d[:, 2, :], torch.ones_like(pts_2d[:, 2, :]))
    proj = pts_2d / div.unsqueeze(1)
    reproj = (proj[:, 0:2, :] - norm_M.reshape(m, 2, -1)).norm(dim=1)
    return torch.where(mask, reproj, hinge_term)[valid].mean()


def esfm_loss_edges(Ps, pts3D, cam, pt, vals, margin, hinge, hinge_w, equalize, valid_only):
    """The same loss and hooked gradients on the E observed pairs only (no [m, 3, n] tensor), so
    the checker also runs at config-4 size; pinned against ``esfm_loss`` in tests/test_oracle.py."""
    w = hinge_w if hinge else 0.0
    y = torch.einsum("eij,je->ei", Ps[cam], pts3D[:, pt])  # [E, 3]
    z = y[:, 2]
    mask = (z >= margin) if hinge else (z.abs() >= margin)
    if equalize and y.requires_grad:
        if valid_only:
            npos = torch.clamp(mask.sum(), min=1).to(y.dtype)
            y.register_hook(lambda g: torch.where(mask[:, None], F.normalize(g, dim=1) / npos, g))
        else:
            y.register_hook(lambda g: F.normalize(g, dim=1) / y.shape[0])
    hinge_term = (margin - y[:, 2]) * w
    div = torch.where(mask, y[:, 2], torch.ones_like(y[:, 2]))
    reproj = (y[:, 0:2] / div[:, None] - vals.to(y.dtype)).norm(dim=1)
    return torch.where(mask, reproj, hinge_term).mean()
