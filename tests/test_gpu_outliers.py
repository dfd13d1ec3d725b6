"""Device outlier injection (gasfm_amd/outliers.py, csrc/outliers.hip) against the reference.

tests/golden/outliers.npz holds the reference's own ``dataset_utils.inject_outliers`` outputs
(make_golden_outliers.py, CPU, fixed seeds).  Bars:
  - selection: bit-exact outlier mask, and numpy's RNG left at the same position (same draws);
  - values for the same Gaussian draws z: |d| <= 1e-5 (|ref| + sqrt(sigma_ii[view])) (fp32
    rounding of the reference's per-view moment sums; see tests/test_outliers_oracle.py);
  - the returned scene: indices bit-exact, normalised values to the same relative bound.
Larger scenes are checked against oracle/outliers.py (mask bit-exact; the oracle's fp64 moments).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from gasfm_amd import synthetic
from gasfm_amd.outliers import OutlierInjector, inject_outliers
from gasfm_amd.scene_device import scene_from_dense_device
from oracle import outliers as O

pytestmark = pytest.mark.gpu
CASES = ["c1_r10", "w_r20", "w_r35", "r_r25", "c1_fail"]


def _edges(M):
    valid = (np.abs(M[0::2]) + np.abs(M[1::2])) != 0
    return np.nonzero(valid)


def _scene(M, Ns, device):
    m = M.shape[0] // 2
    Ps = torch.zeros((m, 3, 4))
    return scene_from_dense_device(torch.from_numpy(M).to(device), torch.from_numpy(Ns).to(device), Ps.to(device))


@pytest.mark.parametrize("tag", CASES)
def test_inject_outliers_matches_reference_fixture(device, tag):
    f = golden("outliers.npz")
    M, Ns = f[tag + "_M"], f[tag + "_Ns"]
    rate, np_seed, _ = f[tag + "_params"]
    data = _scene(M, Ns, device)
    logs = []
    z = torch.from_numpy(f[tag + "_z"]) if not int(f[tag + "_failed"]) else None
    np.random.seed(int(np_seed))
    res = inject_outliers(data, float(rate), z=z, log=logs.append)
    assert np.array_equal(np.random.randint(0, 2**31 - 1, size=4), f[tag + "_np_next"])
    if int(f[tag + "_failed"]):
        assert res is None and len(logs) == 5
        return
    mask = res.outliers_mask.cpu().numpy()
    assert np.array_equal(mask, f[tag + "_mask"])
    cam, pt = _edges(M)
    Mn = res._M.cpu().numpy()
    got = np.stack([Mn[2 * cam, pt], Mn[2 * cam + 1, pt]], 1)
    ref = f[tag + "_pix_out"]
    pix = np.stack([M[2 * cam, pt], M[2 * cam + 1, pt]], 1)
    _, _, sigma, _ = O.inject_values(pix, cam, M.shape[0] // 2, mask, f[tag + "_z"])
    spread = np.sqrt(np.stack([sigma[cam, 0, 0], sigma[cam, 1, 1]], 1))
    assert np.all(np.abs(got - ref) <= 1e-5 * (np.abs(ref) + spread))
    assert np.array_equal(got[~mask], pix[~mask])
    # the returned SceneData: same projections, values normalised by Ns
    assert np.array_equal(res.x.indices.cpu().numpy(), f[tag + "_indices"])
    rv, vref = res.x.values.cpu().numpy(), f[tag + "_values"]
    assert np.all(np.abs(rv - vref) <= 1e-5 * (np.abs(vref) + spread / 800.0) + 1e-7)


@pytest.mark.parametrize("m,n,extra,rate,seed", [(120, 30000, 8, 0.10, 1), (300, 60000, 5, 0.30, 2)])
def test_inject_outliers_matches_oracle_larger(device, m, n, extra, rate, seed):
    sc = synthetic.windowed_scene(m, n, mean_extra=extra, seed=seed)
    M, Ns = sc.dense_M(), sc.Ns()
    cam, pt = _edges(M)
    np.random.seed(seed)
    ref_mask = O.select_outliers(cam, pt, m, n, rate, log=lambda s: None)
    ref_next = np.random.randint(0, 2**31 - 1, size=4)
    np.random.seed(seed)
    inj = OutlierInjector(torch.from_numpy(M).to(device), rate, log=lambda s: None)
    mask = inj.select_outliers()
    assert np.array_equal(np.random.randint(0, 2**31 - 1, size=4), ref_next)
    assert ref_mask is not None and np.array_equal(mask.cpu().numpy(), ref_mask)
    assert inj.n_outliers == round(rate * cam.shape[0])
    z = torch.randn((inj.n_outliers, 2, 1), generator=torch.Generator().manual_seed(seed))
    Mn = inj.inject_outliers(z=z).cpu().numpy()
    pix = np.stack([M[2 * cam, pt], M[2 * cam + 1, pt]], 1)
    new, mu, sigma, L = O.inject_values(pix, cam, m, ref_mask, z.numpy())
    got = np.stack([Mn[2 * cam, pt], Mn[2 * cam + 1, pt]], 1)
    spread = np.sqrt(np.stack([sigma[cam, 0, 0], sigma[cam, 1, 1]], 1))
    assert np.all(np.abs(got - new) <= 2e-6 * (np.abs(new) + spread))
    np.testing.assert_allclose(inj.mu.cpu().numpy(), mu, rtol=1e-6)
    np.testing.assert_allclose(inj.sigma.cpu().numpy(), sigma, rtol=1e-6)
    # inliers per view / per point after the injection meet the reference's minima
    inl = ~ref_mask
    assert np.bincount(cam[inl], minlength=m).min() >= 8 and np.bincount(pt[inl], minlength=n).min() >= 2


def test_moments_ldl_interchange_and_pivots(device):
    """gasfm_outlier_moments vs the oracle's restatement of torch.linalg.ldl_factor, with views whose
    x is ~0.05 y (Bunch-Kaufman interchanges) and outlier edges excluded from the moments."""
    from gasfm_amd import _native
    g = np.random.default_rng(5)
    m, per = 16, 100
    vals = g.uniform(1, 1000, size=(m * per, 2)).astype(np.float32)
    for c in range(4):
        s = slice(c * per, (c + 1) * per)
        vals[s, 0] = 0.05 * vals[s, 1] + g.normal(0, 1, per).astype(np.float32)
    state = np.where(g.random(m * per) < 0.2, 3, 2).astype(np.uint8)
    cam = np.repeat(np.arange(m), per)
    cam_ptr = torch.arange(0, m * per + 1, per, dtype=torch.int32, device=device)
    mu, sigma, tril, piv = _native.outlier_moments(torch.from_numpy(vals).to(device), torch.from_numpy(state).to(device),
                                                  cam_ptr, m)
    _, mu_r, sig_r, L_r = O.inject_values(vals, cam, m, state == 3, np.zeros((int((state == 3).sum()), 2)))
    _, piv_r = O.ldl_scale_tril(sigma.cpu().numpy())
    assert np.array_equal(piv.cpu().numpy(), piv_r)
    assert (piv_r[:4, 0] == 2).all() and (piv_r[4:, 0] == 1).all()
    np.testing.assert_allclose(mu.cpu().numpy(), mu_r, rtol=1e-6)
    np.testing.assert_allclose(sigma.cpu().numpy(), sig_r, rtol=1e-6)
    T = tril.cpu().numpy()
    np.testing.assert_allclose(T @ np.swapaxes(T, 1, 2), sig_r, rtol=1e-4)
    np.testing.assert_allclose(T, L_r, rtol=1e-4, atol=1e-4 * float(np.abs(L_r).max()))


def test_inject_outliers_default_draws_keep_graph(device):
    """Default z (torch.randn on the device, as the reference on a CUDA scene): finite values, the
    outliers changed, every inlier untouched, the same projection graph."""
    sc = synthetic.windowed_scene(60, 8000, mean_extra=6, seed=3)
    data = _scene(sc.dense_M(), sc.Ns(), device)
    np.random.seed(0)
    res = inject_outliers(data, 0.1, log=lambda s: None)
    assert res is not None
    assert torch.equal(res.x.indices, data.x.indices)
    mask = res.outliers_mask
    assert int(mask.sum()) == round(0.1 * data.x.indices.shape[1])
    assert torch.isfinite(res.x.values).all()
    assert torch.equal(res.x.values[~mask], data.x.values[~mask])
    assert (res.x.values[mask] != data.x.values[mask]).any(dim=1).all()
