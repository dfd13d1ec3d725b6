"""CPU restatement of the reference's outlier injection (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module, as the checker of gasfm_amd.outliers (the device path).

Follows code/utils/dataset_utils.py:
  OutlierInjector.__init__ / init_fixed_inliers_and_outliers   :160-172, 253-269
  add_margin_to_outlier_rate / add_margin_to_n_new_outliers    :277-299
  sample_more_outliers                                         :301-305
  blacklist_problematic_outliers                               :307-320
  remove_surplus_outlier_candidates                            :322-337
  select_outliers (retry from scratch, 5 tries)                :339-364
  inject_outliers (per-view moments, LDL -> scale_tril, mu+Lz) :366-433
  inject_outliers(scene_data, rate) (pixel M in, new M out)    :436-461
with constants MIN_N_VIEWS_PER_POINT = 2, MIN_N_POINTS_PER_VIEW = 8 (utils/constants.py:2, 6).

Edges are the coalesced COO order of M2sparse(M, normalize=False): camera-major, points
ascending.  The per-edge partition is one code per edge instead of four boolean masks:
0 fixed inlier, 1 fixed outlier (never set by the reference), 2 free inlier, 3 free outlier.
The random draws are the reference's: numpy's global RNG, ``np.random.choice(idx, size,
replace=False)`` over the sorted nonzero() index list (legacy RandomState: ``permutation(len)[:size]``,
so only the list length matters).  The Gaussian draws ``z`` (torch.randn((n_out, 2, 1)) in the
reference) are an input here.

Pinned by tests/golden/outliers.npz (tests/golden/make_golden_outliers.py: the reference's own
``inject_outliers`` run on CPU scenes with fixed seeds): masks bit-exact, values to fp32 rounding.
"""
import numpy as np

MIN_N_VIEWS_PER_POINT = 2
MIN_N_POINTS_PER_VIEW = 8

FIXED_IN, FIXED_OUT, FREE_IN, FREE_OUT = 0, 1, 2, 3


def _inlier_counts(state, cam, pt, m, n):
    inl = (state & 1) == 0
    return (np.bincount(cam[inl], minlength=m), np.bincount(pt[inl], minlength=n))


def _margin_rate(rate, w=0.5):
    # add_margin_to_outlier_rate (dataset_utils.py:277-283): weighted harmonic mean with 1
    r = 1.0 / (w * 1.0 / rate + (1.0 - w) * 1.0 / 1.0)
    assert 0 < rate < r < 1
    return r


def select_outliers(cam, pt, m, n, rate, n_tries=5, rng=None, log=print):
    """Outlier mask [E] bool (OutlierInjector.select_outliers) or None after n_tries failures."""
    rng = np.random if rng is None else rng
    cam = np.asarray(cam, dtype=np.int64)
    pt = np.asarray(pt, dtype=np.int64)
    E = cam.shape[0]
    assert 0 < rate < 1
    ppv = np.bincount(cam, minlength=m)
    vpp = np.bincount(pt, minlength=n)
    assert np.all(ppv >= MIN_N_POINTS_PER_VIEW)  # verify_enough_points_per_view (:240-244)
    assert np.all(vpp >= MIN_N_VIEWS_PER_POINT)  # verify_enough_views_per_point (:246-251)
    target = round(rate * E)  # target_n_outliers (:224-226), Python's round

    def fresh():  # init_fixed_inliers_and_outliers + init_free_inliers_and_outliers (:253-275)
        fixed = (vpp[pt] < MIN_N_VIEWS_PER_POINT + 1) | (ppv[cam] < MIN_N_POINTS_PER_VIEW + 1)
        return np.where(fixed, FIXED_IN, FREE_IN).astype(np.uint8)

    state = fresh()
    while True:
        if not n_tries > 0:
            return None
        retry = False
        while int(np.sum((state & 1) == 1)) < target:
            n_out = int(np.sum((state & 1) == 1))
            n_free_in = int(np.sum(state == FREE_IN))
            target_new = target - n_out
            if not target_new <= n_free_in:
                state = fresh()
                log('Retry outlier sampling, {} attempts remaining.'.format(n_tries - 1))
                n_tries -= 1
                retry = True
                break
            # add_margin_to_n_new_outliers (:285-299)
            n_new = round(_margin_rate(target_new / n_free_in) * n_free_in)
            assert n_new <= n_free_in
            # sample_more_outliers (:301-305)
            state = _flip(state, FREE_IN, FREE_OUT, n_new, rng)
            # blacklist_problematic_outliers (:307-320)
            cin, pin = _inlier_counts(state, cam, pt, m, n)
            bad = (pin[pt] < MIN_N_VIEWS_PER_POINT) | (cin[cam] < MIN_N_POINTS_PER_VIEW)
            state[(state == FREE_OUT) & bad] = FIXED_IN
        if retry:
            continue
        # remove_surplus_outlier_candidates (:322-337)
        cin, pin = _inlier_counts(state, cam, pt, m, n)
        assert np.all(cin >= MIN_N_POINTS_PER_VIEW) and np.all(pin >= MIN_N_VIEWS_PER_POINT)
        n_out = int(np.sum((state & 1) == 1))
        assert n_out >= target
        state = _flip(state, FREE_OUT, FREE_IN, n_out - target, rng)
        assert int(np.sum((state & 1) == 1)) == target
        cin, pin = _inlier_counts(state, cam, pt, m, n)
        assert np.all(cin >= MIN_N_POINTS_PER_VIEW) and np.all(pin >= MIN_N_VIEWS_PER_POINT)
        return (state & 1) == 1


def _flip(state, frm, to, size, rng):
    """state[nonzero(state == frm)[choice]] = to, one np.random.choice draw (:303, :330)."""
    idx = np.nonzero(state == frm)[0]
    sel = rng.choice(idx, size=(size,), replace=False)
    out = state.copy()
    out[sel] = to
    return out


def ldl_scale_tril(sigma):
    """scale_tril [V, 2, 2] with sigma = L L^T from LAPACK sytf2 (lower, Bunch-Kaufman) as
    inject_outliers uses torch.linalg.ldl_factor (:378-392); pivots [V, 2] (negative: a 2x2
    block, on which the reference's assert fails)."""
    s = np.asarray(sigma, dtype=np.float32)
    V = s.shape[0]
    alpha = np.float32((1.0 + np.sqrt(17.0)) / 8.0)
    L = np.zeros((V, 2, 2), dtype=np.float32)
    piv = np.zeros((V, 2), dtype=np.int32)
    for v in range(V):
        a, b, c = s[v, 0, 0], s[v, 1, 0], s[v, 1, 1]
        colmax = abs(b)
        swap = False
        if abs(a) >= alpha * colmax:
            piv[v] = (1, 2)
        elif abs(c) >= alpha * colmax:
            piv[v] = (2, 2)
            swap = True
            a, c = c, a
        else:
            piv[v] = (-2, -2)
            L[v] = np.nan
            continue
        d11 = np.float32(1.0) / a
        d1 = c + b * ((-d11) * b)
        l10 = d11 * b
        sa, sd = np.sqrt(a), np.sqrt(d1)
        t = np.array([[sa, 0.0], [l10 * sa, sd]], dtype=np.float32)
        L[v] = t[::-1] if swap else t
    return L, piv


def inject_values(values, cam, m, outlier_mask, z):
    """New pixel values [E, 2] (inject_outliers :366-433): per-view mean and Bessel-corrected raw
    second moment of the inliers, scale_tril from the LDL factorisation, outlier k (edge order)
    = mu[cam] + L[cam] z[k].  Accumulates in fp64 (the reference sums fp32 sparse values)."""
    values = np.asarray(values, dtype=np.float32)
    cam = np.asarray(cam, dtype=np.int64)
    out = np.asarray(outlier_mask, dtype=bool)
    inl = ~out
    N = np.bincount(cam[inl], minlength=m).astype(np.float64)
    assert np.all(N >= MIN_N_POINTS_PER_VIEW)
    v = values[inl].astype(np.float64)
    c = cam[inl]
    s = np.stack([np.bincount(c, weights=v[:, 0], minlength=m), np.bincount(c, weights=v[:, 1], minlength=m)], 1)
    sxx = np.bincount(c, weights=v[:, 0] * v[:, 0], minlength=m)
    sxy = np.bincount(c, weights=v[:, 0] * v[:, 1], minlength=m)
    syy = np.bincount(c, weights=v[:, 1] * v[:, 1], minlength=m)
    mu = (s / N[:, None]).astype(np.float32)
    sigma = np.stack([np.stack([sxx, sxy], 1), np.stack([sxy, syy], 1)], 1) / (N - 1)[:, None, None]
    L, piv = ldl_scale_tril(sigma.astype(np.float32))
    assert np.all(piv > 0)
    oc = cam[out]
    zz = np.asarray(z, dtype=np.float32).reshape(-1, 2)
    assert zz.shape[0] == oc.shape[0]
    new = values.copy()
    new[out] = mu[oc] + np.einsum("kij,kj->ki", L[oc].astype(np.float64), zz.astype(np.float64)).astype(np.float32)
    return new, mu, sigma.astype(np.float32), L
