"""Outlier-injection oracle (oracle/outliers.py) against the reference's own outputs.

tests/golden/outliers.npz comes from the reference's ``dataset_utils.inject_outliers`` run on CPU
scenes under fixed numpy / torch seeds (tests/golden/make_golden_outliers.py).  The selection is
integer work and must be bit-exact, including the position of numpy's RNG afterwards (the same
number of draws); the injected pixel values agree to fp32 rounding of the per-view moments (the
reference sums fp32 squares of ~1e3-pixel values over hundreds of inliers per view):
|d| <= 1e-5 (|ref| + sqrt(sigma_ii[view])), sigma = the view's second-moment matrix.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import outliers as O

CASES = ["c1_r10", "w_r20", "w_r35", "r_r25", "c1_fail"]


def _edges(M):
    valid = (np.abs(M[0::2]) + np.abs(M[1::2])) != 0
    cam, pt = np.nonzero(valid)
    return cam, pt


@pytest.mark.parametrize("tag", CASES)
def test_oracle_selection_and_values_match_reference(tag):
    f = golden("outliers.npz")
    M = f[tag + "_M"]
    rate, np_seed, _ = f[tag + "_params"]
    m, n = M.shape[0] // 2, M.shape[1]
    cam, pt = _edges(M)
    logs = []
    np.random.seed(int(np_seed))
    mask = O.select_outliers(cam, pt, m, n, float(rate), log=logs.append)
    assert np.array_equal(np.random.randint(0, 2**31 - 1, size=4), f[tag + "_np_next"])
    if int(f[tag + "_failed"]):
        assert mask is None and len(logs) == 5
        return
    assert np.array_equal(mask, f[tag + "_mask"])
    pix = np.stack([M[2 * cam, pt], M[2 * cam + 1, pt]], 1)
    new, mu, sigma, L = O.inject_values(pix, cam, m, mask, f[tag + "_z"])
    ref = f[tag + "_pix_out"]
    spread = np.sqrt(np.stack([sigma[cam, 0, 0], sigma[cam, 1, 1]], 1))
    assert np.all(np.abs(new - ref) <= 1e-5 * (np.abs(ref) + spread))
    assert np.array_equal(new[~mask], pix[~mask])
    np.testing.assert_allclose(L @ np.swapaxes(L, 1, 2), sigma, rtol=1e-5)


def test_ldl_matches_torch_ldl_factor_including_interchange():
    """oracle.ldl_scale_tril vs the reference's own construction from torch.linalg.ldl_factor
    (dataset_utils.py:378-392), on PSD matrices with and without the row interchange."""
    g = np.random.default_rng(0)
    A = g.normal(size=(64, 2, 2)).astype(np.float32)
    S = A @ np.swapaxes(A, 1, 2) + 1e-3 * np.eye(2, dtype=np.float32)
    # small first diagonal against the off-diagonal: Bunch-Kaufman interchanges rows 1 and 2
    S[:8] = np.stack([np.array([[0.01, 0.08], [0.08, 1.0]], np.float32) * (k + 1) for k in range(8)])
    sigma = torch.from_numpy(S)
    LD, piv = torch.linalg.ldl_factor(sigma)
    Lt = LD.clone()
    Lt[:, [0, 1], [0, 1]] = 1
    D = torch.zeros_like(LD)
    D[:, [0, 1], [0, 1]] = LD[:, [0, 1], [0, 1]]
    T = Lt @ torch.sqrt(D)
    perm = ~((piv[:, 0] == 1) & (piv[:, 1] == 2))
    T[perm] = torch.flip(T[perm], [1])
    L, p = O.ldl_scale_tril(S)
    assert np.array_equal(p, piv.numpy())
    assert perm[:8].all() and not perm[8:].all()
    # MKL orders the sytf2 arithmetic its own way: agreement to fp32 rounding of the 2x2 factors
    np.testing.assert_allclose(L, T.numpy(), rtol=1e-5, atol=2e-6 * float(np.abs(T.numpy()).max()))
