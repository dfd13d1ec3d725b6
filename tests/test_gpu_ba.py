"""Device bundle adjustment (gasfm_amd/ba.py, csrc/bundle_adjust.hip) against oracle/ba.py.

Both sides are fp64 and run the same restated Ceres LM (oracle/ba.py documents it): the device
evaluates residuals / Jacobians with dual numbers and eliminates the points (Schur complement +
rocSOLVER Cholesky), the oracle uses complex-step Jacobians and a dense solve.  Bars: residuals,
Jacobians and one LM step to 1e-9 relative; whole euc_ba / proj_ba runs (two LM solves with a DLT
triangulation between) to 1e-6 relative in the refined cameras / points with the same iteration
counts; the DLT to 1e-8 of the reference's own fixture (tests/golden/ba.npz).  Known answer:
noise-free scenes converge to < 1e-6 px.  Determinism: two runs bitwise identical.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from gasfm_amd import ba as B
from gasfm_amd import synthetic
from oracle import ba as O

pytestmark = pytest.mark.gpu


def _problems(kind, device, noise=0.3):
    sc = synthetic.ba_scene(7, 60, 3, noise_px=noise, seed=11)
    vis = O.valid_points(sc["xs"])
    c, p = np.where(vis)
    obs = sc["xs"][vis]
    rng = np.random.default_rng(12)
    X0 = sc["Xs"] + 0.01 * rng.standard_normal(sc["Xs"].shape)
    if kind == "euc":
        cam0, K = O.euc_camera_params(sc["Rs"], sc["ts"] + 0.02 * rng.standard_normal(sc["ts"].shape), sc["Ks"])
        po = O.Problem("euc", cam0, X0, c, p, obs, K)
        Kd = torch.from_numpy(K).to(device)
    else:
        P = O.camera_matrices(sc["Rs"], sc["ts"], sc["Ks"]).reshape(-1, 12, order="F")
        cam0 = P * (1 + 1e-3 * rng.standard_normal(P.shape))
        po = O.Problem("proj", cam0, X0, c, p, obs)
        Kd = None
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    pd = B.BAProblem(kind, t(cam0), t(X0), t(c), t(p), t(obs), Kd)
    return po, pd


@pytest.mark.parametrize("kind", ["euc", "proj"])
def test_eval_and_jacobians_match_oracle(device, kind):
    po, pd = _problems(kind, device)
    g = np.random.default_rng(1)
    x = 1e-3 * g.standard_normal(po.N)
    dc, dX = po.split(x)
    cost_o, f_o, J_o = po.evaluate(x)
    cost_d = pd.evaluate(torch.from_numpy(dc.copy()).to(device), torch.from_numpy(dX.copy()).to(device), True)
    assert abs(cost_d - cost_o) <= 1e-10 * cost_o
    np.testing.assert_allclose(pd.fres.cpu().numpy().reshape(-1), f_o, rtol=1e-10, atol=1e-12)
    E, CP = po.cidx.shape[0], po.CP
    Jc, Jp = pd.Jc.cpu().numpy(), pd.Jp.cpu().numpy()
    rows = np.arange(E)
    scale = np.abs(J_o).max()
    for i in range(2):
        for k in range(CP):
            np.testing.assert_allclose(Jc[:, i, k], J_o[2 * rows + i, po.cidx * CP + k], rtol=1e-9, atol=1e-12 * scale)
        for k in range(3):
            np.testing.assert_allclose(Jp[:, i, k], J_o[2 * rows + i, po.m * CP + 3 * po.pidx + k], rtol=1e-9,
                                       atol=1e-12 * scale)


@pytest.mark.parametrize("kind", ["euc", "proj"])
def test_schur_step_matches_dense_solve(device, kind):
    po, pd = _problems(kind, device)
    x = np.zeros(po.N)
    _, f, J = po.evaluate(x)
    scale = 1.0 / (1.0 + np.sqrt((J * J).sum(0)))
    Js = J * scale
    radius = 37.0
    diag = np.clip((Js * Js).sum(0), 1e-6, 1e32)
    step = -np.linalg.solve(Js.T @ Js + np.diag(diag / radius), Js.T @ f)
    mr = Js @ step
    model_o = -mr @ (f + mr / 2)
    z = lambda *s: torch.zeros(s, dtype=torch.float64, device=device)  # noqa: E731
    pd.evaluate(z(po.m, po.CP), z(po.n, 3), True)
    pd.normals()
    pd.sc = (1.0 / (1.0 + torch.sqrt(torch.diagonal(pd.U, dim1=1, dim2=2)))).contiguous()
    pd.sp = (1.0 / (1.0 + torch.sqrt(torch.diagonal(pd.V, dim1=1, dim2=2)))).contiguous()
    np.testing.assert_allclose(np.concatenate([pd.sc.cpu().numpy().reshape(-1), pd.sp.cpu().numpy().reshape(-1)]),
                               scale, rtol=1e-10)
    pd.evaluate(z(po.m, po.CP), z(po.n, 3), True)
    pd.normals()
    dc, dp = pd.step(radius)
    got = np.concatenate([dc.cpu().numpy().reshape(-1), dp.cpu().numpy().reshape(-1)])
    np.testing.assert_allclose(got, step, rtol=1e-8, atol=1e-10 * np.abs(step).max())
    assert abs(pd.model_change(dc, dp) - model_o) <= 1e-8 * abs(model_o)


def test_dlt_matches_reference_fixture(device):
    f = golden("ba.npz")
    xs = torch.from_numpy(f["xs"]).to(device)
    ed = B._Edges(xs)
    X = ed.dlt(torch.from_numpy(f["Ps"]).to(device), torch.from_numpy(np.linalg.inv(f["Ks"])).to(device)).cpu().numpy()
    ref = f["X_dlt"]
    assert np.array_equal(np.isnan(X), np.isnan(ref))
    np.testing.assert_allclose(X, ref, rtol=1e-8, atol=1e-10)
    Ps = torch.from_numpy(f["Ps"]).to(device)
    ref_err = np.nanmean(f["err_dlt"])
    assert abs(ed.repro(Ps, torch.from_numpy(ref).to(device)) - ref_err) <= 1e-12 * ref_err


def _cmp(got, ref, keys, rtol):
    for k in keys:
        np.testing.assert_allclose(got[k], ref[k], rtol=rtol, atol=rtol * max(1.0, float(np.nanmax(np.abs(ref[k])))),
                                   err_msg=k)


def test_euc_ba_matches_oracle(device):
    sc = synthetic.ba_scene(9, 90, 4, noise_px=0.5, seed=21)
    rng = np.random.default_rng(22)
    Rs = np.stack([O.rodrigues_to_matrix(O.matrix_to_rodrigues(R) + 0.01 * rng.standard_normal(3)) for R in sc["Rs"]])
    ts = sc["ts"] + 0.03 * rng.standard_normal(sc["ts"].shape)
    Xs = sc["Xs"] + 0.02 * rng.standard_normal(sc["Xs"].shape)
    ref = O.euc_ba(sc["xs"], Rs, ts, sc["Ks"], Xs_our=Xs, repeat=True)
    got = B.euc_ba(sc["xs"], Rs, ts, sc["Ks"], Xs_our=Xs, repeat=True, print_out=False)
    for s in ("summary1", "summary2"):
        assert got[s]["iterations"] == ref[s]["iterations"] and got[s]["termination"] == ref[s]["termination"]
        np.testing.assert_allclose(got[s]["costs"], ref[s]["costs"], rtol=1e-8)
    _cmp(got, ref, ("Rs", "ts", "Ps", "Xs"), 1e-6)
    for k in ("repro_before", "repro_middle", "repro_middle_triangulated", "repro_after"):
        assert abs(got[k] - ref[k]) <= 1e-7 * ref[k], k
    assert got["repro_after"] < got["repro_before"]


def test_proj_ba_matches_oracle(device):
    sc = synthetic.ba_scene(8, 80, 4, noise_px=0.5, seed=31)
    Ps = O.camera_matrices(sc["Rs"], sc["ts"], sc["Ks"])
    rng = np.random.default_rng(32)
    Ps_p = Ps * (1 + 1e-3 * rng.standard_normal(Ps.shape))
    Xs = sc["Xs"] + 0.02 * rng.standard_normal(sc["Xs"].shape)
    Ns = np.linalg.inv(sc["Ks"])
    ref = O.proj_ba(Ps_p, sc["xs"], Xs_our=Xs, Ns=Ns, repeat=True)
    got = B.proj_ba(Ps_p, sc["xs"], Xs_our=Xs, Ns=Ns, repeat=True, print_out=False)
    for s in ("summary1", "summary2"):
        assert got[s]["iterations"] == ref[s]["iterations"]
        np.testing.assert_allclose(got[s]["costs"], ref[s]["costs"], rtol=1e-8)
    _cmp(got, ref, ("Ps", "Xs"), 1e-6)


def test_noise_free_known_answer_and_triangulation_start(device):
    sc = synthetic.ba_scene(12, 200, 5, noise_px=0.0, seed=41)
    rng = np.random.default_rng(42)
    Rs = np.stack([O.rodrigues_to_matrix(O.matrix_to_rodrigues(R) + 0.01 * rng.standard_normal(3)) for R in sc["Rs"]])
    ts = sc["ts"] + 0.03 * rng.standard_normal(sc["ts"].shape)
    got = B.euc_ba(sc["xs"], Rs, ts, sc["Ks"], triangulation=True, repeat=True, print_out=False)
    assert got["repro_before"] > 1.0 and got["repro_after"] < 1e-6
    assert got["converged1"] and got["converged2"]


def test_larger_scene_converges_deterministically(device):
    sc = synthetic.ba_scene(40, 4000, 6, noise_px=0.5, seed=51)
    rng = np.random.default_rng(52)
    Rs = np.stack([O.rodrigues_to_matrix(O.matrix_to_rodrigues(R) + 0.005 * rng.standard_normal(3)) for R in sc["Rs"]])
    ts = sc["ts"] + 0.02 * rng.standard_normal(sc["ts"].shape)
    Xs = sc["Xs"] + 0.01 * rng.standard_normal(sc["Xs"].shape)
    a = B.euc_ba(sc["xs"], Rs, ts, sc["Ks"], Xs_our=Xs, repeat=True, print_out=False)
    b = B.euc_ba(sc["xs"], Rs, ts, sc["Ks"], Xs_our=Xs, repeat=True, print_out=False)
    for k in ("Rs", "ts", "Xs"):
        assert np.array_equal(a[k], b[k]), k
    assert a["repro_after"] < a["repro_middle"] < a["repro_before"]
    assert a["repro_after"] < 0.6  # 0.5 px noise: the refined error sits at the noise level
    costs = a["summary1"]["costs"]
    assert all(c1 <= c0 for c0, c1 in zip(costs, costs[1:]))
