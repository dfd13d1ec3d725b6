"""Generate tests/golden/core_errors.npz from the REFERENCE's own compute_core_errors (build container only).

    python tests/golden/make_golden_repro.py

Imports code/evaluation.py in place (tests/golden/refimport.py; PyCeres, the bundle-adjustment
binding evaluation.py imports through utils/ba_functions.py, is absent offline and stubbed: the
"our_repro" path does not touch it) and runs ``compute_core_errors(data, pred_dict, conf)`` on the
config-1 scene (the reference SceneData supplies M and Ns_invT) with synthetic float32 predictions
(cameras near identity, points at depths 1.5..6 with homogeneous weights != 1 so pflat matters).
Saved: M, Ns, Ps_norm, pts3D, cam, pt (edges, cam-major), our_repro, and errors at the edges
(from geo_utils.reprojection_error_with_points, the function compute_core_errors averages).
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refimport  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402  (input generation only)


def predictions(m, n, seed=11):
    g = torch.Generator().manual_seed(seed)
    Ps = torch.zeros((m, 3, 4))
    Ps[:, :, :3] = torch.eye(3) + 0.05 * torch.randn((m, 3, 3), generator=g)
    Ps[:, :, 3] = 0.2 * torch.randn((m, 3), generator=g)
    X = torch.randn((3, n), generator=g)
    X[2] = 1.5 + 4.5 * torch.rand(n, generator=g)
    w = 0.5 + torch.rand(n, generator=g)
    return Ps, torch.cat([X * w, w[None]])


def main():
    sys.modules["PyCeres"] = types.ModuleType("PyCeres")
    ref = refimport.load()
    import importlib
    evaluation = importlib.import_module("evaluation")
    geo_utils = importlib.import_module("utils.geo_utils")
    sc = synthetic.config1()
    M, Ns = torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns())
    data = ref.SceneData.SceneData(M, Ns, torch.from_numpy(sc.Ps_gt()), "synthetic_config1", calibrated=True)
    m, n = data.x.shape[0], data.x.shape[1]
    Ps_norm, pts3D = predictions(m, n)
    conf = refimport.DictConf({"dataset": {"calibrated": True},
                               "model": {"view_head": {"enabled": True}, "scenepoint_head": {"enabled": True}},
                               "eval": {"calc_reprojerr_with_gtposes_for_depth_pred": False}})
    core = evaluation.compute_core_errors(data, {"Ps_norm": Ps_norm, "pts3D": pts3D}, conf)
    Ps = data.Ns_invT.transpose(1, 2).numpy() @ Ps_norm.numpy()
    errors = geo_utils.reprojection_error_with_points(Ps, geo_utils.pflat(pts3D).numpy().T,
                                                      geo_utils.M_to_xs(data.M.numpy()))
    cam, pt = data.x.indices[0].numpy(), data.x.indices[1].numpy()
    print("our_repro", core["our_repro"], "edges", cam.shape[0])
    path = os.path.join(HERE, "core_errors.npz")
    np.savez_compressed(path, M=data.M.numpy(), Ns=Ns.numpy(), Ps_norm=Ps_norm.numpy(), pts3D=pts3D.numpy(),
                        cam=cam, pt=pt, our_repro=np.float64(core["our_repro"]), edge_errors=errors[cam, pt])
    print("wrote", path)


if __name__ == "__main__":
    main()
