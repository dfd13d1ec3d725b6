"""compute_core_errors' "our_repro" on the device (gasfm_reproj_error) vs the reference.

Pinned by tests/golden/core_errors.npz (the reference's own compute_core_errors on config 1,
make_golden_repro.py) and by oracle/repro.py (checked against that fixture on the CPU) on a
larger random scene with NaN projections (a point at the origin of homogeneous space).
Tolerance: fp32 projection + division; per-edge rtol 1e-4, mean rtol 2e-5.
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


class _Conf:
    def __init__(self, d):
        self.d = d

    def get_bool(self, key, default=None):
        return self.d.get(key, default)


CONF = _Conf({"model.view_head.enabled": True, "model.scenepoint_head.enabled": True,
              "eval.calc_reprojerr_with_gtposes_for_depth_pred": False})


def test_core_errors_match_reference_fixture(device):
    import gasfm_amd
    from gasfm_amd import evaluation
    f = golden("core_errors.npz")
    data = gasfm_amd.SceneData(torch.from_numpy(f["M"]), torch.from_numpy(f["Ns"]), None, "config1").to(device)
    pred = {"Ps_norm": torch.from_numpy(f["Ps_norm"]).to(device), "pts3D": torch.from_numpy(f["pts3D"]).to(device)}
    assert np.array_equal(data.x.indices[0].cpu().numpy(), f["cam"])
    out = evaluation.compute_core_errors(data, pred, CONF)
    np.testing.assert_allclose(out["our_repro"], f["our_repro"], rtol=2e-5)
    mean, err = evaluation.reprojection_error_mean(data, pred, per_edge=True)
    np.testing.assert_allclose(err.cpu().numpy(), f["edge_errors"], rtol=1e-4, atol=1e-3)


def test_core_errors_match_oracle_random_scene(device):
    import gasfm_amd
    from gasfm_amd import evaluation
    from oracle import repro
    rng = np.random.default_rng(3)
    m, n = 40, 3000
    vis = rng.random((m, n)) < 0.15
    M = (rng.uniform(1, 1000, size=(m, 2, n)) * vis[:, None, :]).reshape(2 * m, n).astype(np.float32)
    K = np.array([[700, 0, 480], [0, 700, 360], [0, 0, 1]])
    Ns = np.repeat(np.linalg.inv(K)[None], m, 0).astype(np.float32)
    Ps = np.zeros((m, 3, 4), dtype=np.float32)
    Ps[:, :, :3] = np.eye(3) + 0.05 * rng.standard_normal((m, 3, 3))
    Ps[:, :, 3] = 0.2 * rng.standard_normal((m, 3))
    X = rng.standard_normal((4, n)).astype(np.float32)
    X[2] = 2 + 3 * rng.random(n)
    X[3] = 0.5 + rng.random(n)
    X[:, 5] = 0.0  # 0/0 -> NaN errors for every edge of point 5 (dropped by nanmean)
    err_ref, mean_ref = repro.reprojection_errors(M.astype(np.float64), Ns.astype(np.float64),
                                                  Ps.astype(np.float64), X.astype(np.float64))
    data = gasfm_amd.SceneData(torch.from_numpy(M), torch.from_numpy(Ns), None, "rand").to(device)
    pred = {"Ps_norm": torch.from_numpy(Ps).to(device), "pts3D": torch.from_numpy(X).to(device)}
    mean, err = evaluation.reprojection_error_mean(data, pred, per_edge=True)
    idx = data.x.indices.cpu().numpy()
    e_ref = err_ref[idx[0], idx[1]]
    assert np.isnan(e_ref).sum() > 0
    np.testing.assert_array_equal(np.isnan(err.cpu().numpy()), np.isnan(e_ref))
    ok = ~np.isnan(e_ref)
    np.testing.assert_allclose(err.cpu().numpy()[ok], e_ref[ok], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(float(mean), mean_ref, rtol=2e-5)
