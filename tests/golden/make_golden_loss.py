"""Generate tests/golden/esfm_loss.npz from the REFERENCE's own ESFMLoss (build container only).

    python tests/golden/make_golden_loss.py

Imports code/loss_functions.py and datasets/SceneData.py in place (tests/golden/refimport.py)
and runs ``ESFMLoss(conf).forward(pred_dict, data)`` + backward in float64 on the config-1 scene
(the reference SceneData supplies norm_M, valid_pts and x.values) with synthetic predictions:
cameras [R | t] near identity, points with depths spread across zero so every branch (valid
depth / hinge / |z| < margin) is hit.  The reference asserts ``data.valid_pts.is_cuda``
(loss_functions.py:122) only to avoid a CPU nonzero bug; the mask is passed as a CPU tensor
whose ``is_cuda`` reads True so the unmodified reference runs on the CPU.

Variants (margin, equalize, valid_only, hinge, hinge_w, dloss):
  v0  1e-4  T T T 1.0  1.0   (conf/learning loss section)
  v1  1e-4  T F T 1.0  1.0   (original normalisation by #valid)
  v2  0.5   F - T 0.7  1.0   (no hook)
  v3  0.5   T T F -    1.0   (no hinge: |z| >= margin)
  v4  1e-4  T T T 1.0 -2.5   (upstream gradient != 1)
Saved: cam, pt, values (edges, cam-major), m, n, Ps, pts3D (fp64 inputs), per variant the
loss, dPs [m, 3, 4], dpts3D [4, n].
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refimport  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402  (input generation only)

VARIANTS = (
    (1e-4, True, True, True, 1.0, 1.0),
    (1e-4, True, False, True, 1.0, 1.0),
    (0.5, False, False, True, 0.7, 1.0),
    (0.5, True, True, False, 0.0, 1.0),
    (1e-4, True, True, True, 1.0, -2.5),
)


class _CpuMaskTaggedCuda(torch.Tensor):
    @property
    def is_cuda(self):
        return True


def predictions(m, n, seed=7):
    g = torch.Generator().manual_seed(seed)
    Ps = torch.zeros((m, 3, 4), dtype=torch.float64)
    Ps[:, :, :3] = torch.eye(3, dtype=torch.float64) + 0.1 * torch.randn((m, 3, 3), generator=g, dtype=torch.float64)
    Ps[:, :, 3] = 0.3 * torch.randn((m, 3), generator=g, dtype=torch.float64)
    X = torch.randn((3, n), generator=g, dtype=torch.float64)
    X[2] = 2.0 + 1.5 * torch.randn(n, generator=g, dtype=torch.float64)
    pts3D = torch.cat([X, torch.ones((1, n), dtype=torch.float64)])
    return Ps, pts3D


def main():
    ref = refimport.load()
    sc = synthetic.config1()
    M, Ns = torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns())
    data = ref.SceneData.SceneData(M, Ns, torch.from_numpy(sc.Ps_gt()), "synthetic_config1", calibrated=True)
    m, n = data.x.shape[0], data.x.shape[1]
    Ps0, X0 = predictions(m, n)
    feed = type("Data", (), {})()
    feed.norm_M = data.norm_M.double()
    feed.valid_pts = data.valid_pts.as_subclass(_CpuMaskTaggedCuda)
    out = {"cam": data.x.indices[0], "pt": data.x.indices[1], "values": data.x.values, "m": m, "n": n,
           "Ps": Ps0, "pts3D": X0, "variants": np.array(VARIANTS, dtype=np.float64)}
    for i, (margin, eq, vo, hinge, w, dloss) in enumerate(VARIANTS):
        conf = refimport.DictConf({"model": {"view_head": {"enabled": True}, "scenepoint_head": {"enabled": True}},
                                   "loss": {"infinity_pts_margin": margin,
                                            "pts_grad_equalization_pre_perspective_divide": eq,
                                            "normalize_grad_wrt_valid_projections_only": vo, "hinge_loss": hinge,
                                            "hinge_loss_weight": w}})
        Ps, X = Ps0.clone().requires_grad_(True), X0.clone().requires_grad_(True)
        loss = ref.loss_functions.ESFMLoss(conf)({"Ps_norm": Ps, "pts3D": X}, feed).as_subclass(torch.Tensor)
        (loss * dloss).backward()
        pos = (Ps0 @ X0)[:, 2, :]
        pos = (pos >= margin) if hinge else (pos.abs() >= margin)
        print(f"v{i}: loss {loss.item():.6f}, valid-depth edges {int((pos & data.valid_pts).sum())} / "
              f"{int(data.valid_pts.sum())}")
        out[f"v{i}_loss"], out[f"v{i}_dPs"], out[f"v{i}_dpts3D"] = loss.detach(), Ps.grad, X.grad
    path = os.path.join(HERE, "esfm_loss.npz")
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in out.items()})
    print("wrote", path)


if __name__ == "__main__":
    main()
