"""Bundle-adjustment oracle (oracle/ba.py): geometry pinned to the reference's own numpy helpers,
the restated Ceres LM pinned by known answers.

tests/golden/ba.npz (make_golden_ba.py) holds the reference's geo_utils outputs on a synthetic
scene: camera matrices, normalisation, DLT triangulation and reprojection errors -- bit-exact
here (same numpy operations).  The Ceres solve itself is absent offline ("parity unpinned"); the
restated solver is checked on noise-free scenes (it must drive the reprojection error to ~0 from
perturbed cameras and points) and on complex-step vs finite-difference Jacobians.
"""
import numpy as np
import pytest

from conftest import golden
from gasfm_amd import synthetic
from oracle import ba as O


def test_geometry_matches_reference_fixture():
    f = golden("ba.npz")
    vis = O.valid_points(f["xs"])
    assert np.array_equal(vis, f["vis"])
    Ps = O.camera_matrices(f["Rs"], f["ts"], f["Ks"])
    assert np.array_equal(Ps, f["Ps"])
    nP, nx = O.normalize_points_cams(Ps, f["xs"], np.linalg.inv(f["Ks"]))
    assert np.array_equal(nP, f["norm_P"]) and np.array_equal(nx, f["norm_x"])
    X = O.dlt_triangulation(nP, nx, vis)
    assert np.array_equal(np.isnan(X), np.isnan(f["X_dlt"]))
    np.testing.assert_allclose(X, f["X_dlt"], rtol=1e-12, atol=1e-12)
    e = O.reprojection_errors(Ps, X, f["xs"], vis)
    np.testing.assert_allclose(e, f["err_dlt"], rtol=1e-10, atol=1e-12)
    e = O.reprojection_errors(Ps, np.concatenate([f["X_gt"], np.ones((f["X_gt"].shape[0], 1))], 1), f["xs"], vis)
    np.testing.assert_allclose(e, f["err_gt"], rtol=1e-10, atol=1e-12)


def _perturbed(sc, seed, rot=0.01, trans=0.03, pts=0.02):
    rng = np.random.default_rng(seed)
    Rs = np.stack([O.rodrigues_to_matrix(O.matrix_to_rodrigues(R) + rot * rng.standard_normal(3)) for R in sc["Rs"]])
    return Rs, sc["ts"] + trans * rng.standard_normal(sc["ts"].shape), sc["Xs"] + pts * rng.standard_normal(sc["Xs"].shape)


def test_rodrigues_roundtrip_and_ceres_rotation():
    g = np.random.default_rng(0)
    for r in list(g.normal(size=(20, 3))) + [np.array([np.pi - 1e-7, 0, 0]), np.array([1e-12, 0, 0])]:
        R = O.rodrigues_to_matrix(r)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
        np.testing.assert_allclose(O.rodrigues_to_matrix(O.matrix_to_rodrigues(R)), R, atol=1e-8)
        p = g.normal(size=3)
        np.testing.assert_allclose(O.angle_axis_rotate_point(r, p), R @ p, atol=1e-12)


@pytest.mark.parametrize("kind", ["euc", "proj"])
def test_complex_step_jacobian_matches_finite_differences(kind):
    sc = synthetic.ba_scene(6, 40, 3, seed=3)
    vis = O.valid_points(sc["xs"])
    c, p = np.where(vis)
    if kind == "euc":
        cam0, K = O.euc_camera_params(sc["Rs"], sc["ts"], sc["Ks"])
        prob = O.Problem("euc", cam0, sc["Xs"], c, p, sc["xs"][vis] + 0.3, K)
    else:
        Ps = O.camera_matrices(sc["Rs"], sc["ts"], sc["Ks"])
        prob = O.Problem("proj", Ps.reshape(-1, 12, order="F"), sc["Xs"], c, p, sc["xs"][vis] + 0.3)
    x = 1e-3 * np.random.default_rng(4).standard_normal(prob.N)
    _, f, J = prob.evaluate(x)
    # Ceres' Huber corrector scales the Jacobian by w = sqrt(rho'): undo it, compare with the
    # central difference of the raw residuals
    w = np.repeat(np.sqrt(O.huber((prob.residuals(x) ** 2).sum(-1))[1]), 2)
    Jr = J / w[:, None]
    h = 1e-6
    for k in np.random.default_rng(5).choice(prob.N, 12, replace=False):
        e = np.zeros(prob.N)
        e[k] = h
        fd = ((prob.residuals(x + e) - prob.residuals(x - e)) / (2 * h)).reshape(-1)
        np.testing.assert_allclose(Jr[:, k], fd, rtol=1e-5, atol=1e-6 * np.abs(Jr).max())


def test_euc_ba_noise_free_converges_to_zero():
    sc = synthetic.ba_scene(10, 120, 4, noise_px=0.0, seed=1)
    Rs, ts, Xs = _perturbed(sc, 2)
    r = O.euc_ba(sc["xs"], Rs, ts, sc["Ks"], Xs_our=Xs, repeat=True)
    assert r["repro_before"] > 1.0
    assert r["repro_after"] < 1e-6 and r["converged1"] and r["converged2"]
    assert r["summary2"]["termination"] == "CONVERGENCE"


def test_proj_ba_noise_free_converges_to_zero():
    sc = synthetic.ba_scene(8, 100, 4, noise_px=0.0, seed=6)
    Ps = O.camera_matrices(sc["Rs"], sc["ts"], sc["Ks"])
    rng = np.random.default_rng(7)
    Ps_p = Ps * (1 + 1e-3 * rng.standard_normal(Ps.shape))
    Xs = sc["Xs"] + 0.02 * rng.standard_normal(sc["Xs"].shape)
    r = O.proj_ba(Ps_p, sc["xs"], Xs_our=Xs, Ns=np.linalg.inv(sc["Ks"]), repeat=True)
    assert r["repro_before"] > 0.5 and r["repro_after"] < 1e-6
