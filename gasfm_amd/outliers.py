"""Outlier injection on the device (BASELINE config 5's per-sample transform).

The reference's ``dataset_utils.inject_outliers(scene_data, rate)`` (utils/dataset_utils.py:436-461,
called per training sample at train.py:73-81) replaces a fraction ``rate`` of the projections by
draws from a per-view bivariate Gaussian fitted to the inliers, choosing them so that every view
keeps >= 8 and every point >= 2 inlier projections.  It works on torch sparse COO tensors and
re-coalesces / re-sums them in every round of its selection loop.

Here the E projections stay in M2sparse's camera-major order on the device, with one class byte
per edge (0 fixed inlier, 2 free inlier, 3 free outlier; 1 = fixed outlier is never produced),
and every pass over them is a HIP kernel (csrc/outliers.hip):

  reference step (dataset_utils.py)          here
  -----------------------------------------  ---------------------------------------------------
  M2sparse(M, normalize=False)     :441      gasfm_scene_mask / _emit / _point_csr (scene_build)
  init_fixed_inliers_and_outliers  :253-269  gasfm_outlier_mark mode 0
  sample_more_outliers             :301-305  np.random.choice on the host (same numpy draw), the
                                             chosen ranks flipped through torch.nonzero's list
  blacklist_problematic_outliers   :307-320  gasfm_outlier_counts + gasfm_outlier_mark mode 1
  remove_surplus_outlier_candidates:322-337  np.random.choice + flip, gasfm_outlier_counts checks
  sparse_moment_estimation + LDL  :366-392   gasfm_outlier_moments (one wave per view)
  mu + scale_tril @ randn          :397-400  gasfm_outlier_apply into a copy of the dense M
  SceneData(M, Ns, ...)            :452-461  scene_from_dense_device (the device graph build)

The selection is bit-identical to the reference's for the same numpy seed (the draws are the
reference's own ``np.random.choice`` calls, in order; only the list lengths reach the host), and
the injected values agree to fp32 rounding for the same Gaussian draws ``z``
(tests/golden/outliers.npz, made by the reference's code).  Host syncs: the four class counts
after every marking pass (the loop is data-dependent and the numpy draw sizes depend on them),
one for the initial counts and minima, and one for all deferred checks at the end; a selection is
flipped by its ranks (a cumulative count over the class, no nonzero() list), the checks between
passes (the reference's verify_* asserts) are collected on the device and tested once.
"""
import numpy as np
import torch

from . import _native
from .scene import MIN_N_POINTS_PER_VIEW, MIN_N_VIEWS_PER_POINT
from .scene_device import _dense_M, scene_from_dense_device

FIXED_IN, FIXED_OUT, FREE_IN, FREE_OUT = 0, 1, 2, 3


class OutlierInjector:
    """dataset_utils.OutlierInjector (:159-433) over the projections of a dense pixel matrix M on
    the device.  ``rng``: the numpy generator of the draws (default: numpy's global RNG, as the
    reference); ``log``: the sink of the reference's retry message."""

    def __init__(self, M, outlier_injection_rate, rng=None, log=print):
        assert 0 < outlier_injection_rate < 1
        if not M.is_cuda:
            raise TypeError("OutlierInjector: M must be a CUDA tensor (no CPU fallback)")
        self.M = M.contiguous()
        self.rate = outlier_injection_rate
        self.rng = np.random if rng is None else rng
        self.log = log
        self.n_views, self.n_points = M.shape[0] // 2, M.shape[1]
        b = _native.scene_build(self.M)  # M2sparse(M, normalize=False): pixel values, cam-major
        self.cam, self.pt, self.values = b["cam"], b["pt"], b["values"]
        self.cam_ptr, self.pt_ptr, self.perm = b["cam_ptr"], b["pt_ptr"], b["perm"]
        self.state = torch.empty(self.cam.shape[0], dtype=torch.uint8, device=M.device)
        self.counts = [0, 0, 0, 0]
        self._checks = []  # [views min, points min] inlier-count minima, tested once (_run_checks)
        self._all_cam = (self.cam_ptr[1:] - self.cam_ptr[:-1]).contiguous()
        self._all_pt = (self.pt_ptr[1:] - self.pt_ptr[:-1]).contiguous()
        # verify_enough_points_per_view / verify_enough_views_per_point (:240-251) and the initial
        # partition's counts in one host read
        c = _native.outlier_mark(self.state, self.cam, self.pt, self._all_cam, self._all_pt, 0)
        if self.n_proj_total:
            mins = torch.stack([self._all_cam.min(), self._all_pt.min()]).to(c.dtype)
            vals = torch.cat([mins, c.view(-1)]).tolist()
        else:
            vals = [0, 0] + c.view(-1).tolist()
        assert vals[0] >= MIN_N_POINTS_PER_VIEW and vals[1] >= MIN_N_VIEWS_PER_POINT
        self.counts = [int(v) for v in vals[2:]]

    # ---- counts (the reference's n_* properties, :182-226)
    @property
    def n_proj_total(self):
        return int(self.cam.shape[0])

    @property
    def n_outliers(self):
        return self.counts[FIXED_OUT] + self.counts[FREE_OUT]

    @property
    def n_inliers(self):
        return self.counts[FIXED_IN] + self.counts[FREE_IN]

    @property
    def n_free_inliers(self):
        return self.counts[FREE_IN]

    @property
    def n_free_outliers(self):
        return self.counts[FREE_OUT]

    @property
    def target_n_outliers(self):
        return round(self.rate * self.n_proj_total)

    @property
    def outliers_mask(self):
        return (self.state & 1) == 1

    # ---- passes
    def _set_counts(self, c):
        self.counts = [int(v) for v in c.tolist()]

    def _init_partition(self):
        # init_fixed_inliers_and_outliers + init_free_inliers_and_outliers (:253-275)
        self._set_counts(_native.outlier_mark(self.state, self.cam, self.pt, self._all_cam, self._all_pt, 0))

    def _inlier_counts(self):
        cam_in, pt_in, mins = _native.outlier_counts(self.state, self.cam_ptr, self.pt_ptr, self.perm,
                                                     self.n_views, self.n_points)
        return cam_in, pt_in, mins

    def _flip(self, frm, to, size):
        """state[nonzero(state == frm)[np.random.choice(...)]] = to (:303, :330): one numpy draw.
        The k-th edge of class frm (edge order, as nonzero lists them) has rank k = its inclusive
        running count - 1; the edges whose rank was drawn flip -- no host sync."""
        pop = self.counts[frm]
        sel = self.rng.choice(pop, size=(size,), replace=False)
        if size:
            dev = self.state.device
            cls = self.state == frm
            rank = torch.cumsum(cls, 0, dtype=torch.int32).sub_(1).clamp_(min=0).long()
            chosen = torch.zeros(pop, dtype=torch.bool, device=dev)
            sel_t = torch.from_numpy(np.asarray(sel, dtype=np.int64)).pin_memory().to(dev, non_blocking=True)
            chosen[sel_t] = True
            self.state.masked_fill_(cls & chosen[rank], to)
            self.counts[frm] -= size
            self.counts[to] += size

    def _verify_inliers(self):
        # verify_enough_points_per_view / _views_per_point on the remaining inliers (:322-324,
        # :336-337): recorded on the device, tested once by _run_checks
        _, _, mins = self._inlier_counts()
        self._checks.append(mins)

    def _run_checks(self, extra=None):
        """The deferred verify_* asserts in one host read; extra: a tensor whose entries must all be > 0."""
        has_mins = bool(self._checks)
        parts = [torch.stack(self._checks).to(torch.int64).min(0).values] if has_mins else []
        if extra is not None:
            parts.append(extra.to(torch.int64).view(-1))
        self._checks = []
        if not parts:
            return
        v = torch.cat(parts).tolist()
        if has_mins:
            assert v[0] >= MIN_N_POINTS_PER_VIEW and v[1] >= MIN_N_VIEWS_PER_POINT
            v = v[2:]
        assert all(x > 0 for x in v), ("outlier injection: a view lost too many inliers, the LDL needed a 2x2 pivot, or the outlier "
                                    "count drifted from the device mask")

    def sample_more_outliers(self, n_new_outliers):
        self._flip(FREE_IN, FREE_OUT, n_new_outliers)

    def blacklist_problematic_outliers(self):
        cam_in, pt_in, _ = self._inlier_counts()
        self._set_counts(_native.outlier_mark(self.state, self.cam, self.pt, cam_in, pt_in, 1))

    def remove_surplus_outlier_candidates(self):
        self._verify_inliers()
        assert self.n_outliers >= self.target_n_outliers
        assert self.n_free_outliers >= self.n_outliers - self.target_n_outliers
        self._flip(FREE_OUT, FREE_IN, self.n_outliers - self.target_n_outliers)
        assert self.n_outliers == self.target_n_outliers
        self._verify_inliers()

    @staticmethod
    def add_margin_to_outlier_rate(outlier_injection_rate, w_desired=0.5):
        rate_with_margin = 1.0 / (w_desired * 1.0 / outlier_injection_rate + (1.0 - w_desired) * 1.0 / 1.0)
        assert 0 < outlier_injection_rate < rate_with_margin < 1
        return rate_with_margin

    def add_margin_to_n_new_outliers(self, target_n_new_outliers, w_desired=0.5):
        assert target_n_new_outliers <= self.n_free_inliers
        assert 0 < w_desired < 1
        r = self.add_margin_to_outlier_rate(target_n_new_outliers / self.n_free_inliers, w_desired)
        n = round(r * self.n_free_inliers)
        assert n <= self.n_free_inliers
        return n

    def select_outliers(self, n_tries=5):
        """Outlier mask [E] (bool, device) or None when n_tries attempts ran out of free inliers."""
        while True:
            if not n_tries > 0:
                return None
            retry = False
            while self.n_outliers < self.target_n_outliers:
                target_new = self.target_n_outliers - self.n_outliers
                if not target_new <= self.n_free_inliers:
                    self._init_partition()
                    self.log('Retry outlier sampling, {} attempts remaining.'.format(n_tries - 1))
                    n_tries -= 1
                    retry = True
                    break
                self.sample_more_outliers(self.add_margin_to_n_new_outliers(target_new, w_desired=0.5))
                self.blacklist_problematic_outliers()
            if retry:
                continue
            assert self.n_outliers >= self.target_n_outliers
            self.remove_surplus_outlier_candidates()
            self._run_checks()
            return self.outliers_mask

    def inject_outliers(self, z=None, generator=None):
        """Dense pixel matrix with the outliers replaced by mu + scale_tril z (:366-433).
        z [n_out, 2(, 1)]: the Gaussian draws (default torch.randn on M's device, as the
        reference draws on the scene's device)."""
        dev = self.M.device
        mu, sigma, tril, piv = _native.outlier_moments(self.values, self.state, self.cam_ptr, self.n_views)
        _, _, mins = self._inlier_counts()
        n_out = self.n_outliers
        mask = self.outliers_mask
        # :375 (>= 8 inliers per view), the LDL's 1x1 pivots (dataset_utils.py:383) and the host
        # outlier count agreeing with the device mask (nonzero_static below would silently truncate
        # or pad with -1 otherwise), one host read
        self._run_checks(extra=torch.stack([(mins[0] >= MIN_N_POINTS_PER_VIEW).to(torch.int64),
                                            (piv > 0).all().to(torch.int64),
                                            (mask.sum() == n_out).to(torch.int64)]))
        idx = torch.nonzero_static(mask, size=n_out).view(-1)
        if z is None:
            z = torch.randn((n_out, 2, 1), device=dev, generator=generator)
        z = z.to(dev, torch.float32).reshape(n_out, 2).contiguous()
        M_new = self.M.clone()
        _native.outlier_apply(idx, self.cam, self.pt, z, mu, tril, M_new)
        self.mu, self.sigma, self.scale_tril = mu, sigma, tril
        return M_new


def inject_outliers(scene_data, outlier_injection_rate, z=None, generator=None, rng=None, log=print, max_piece=None):
    """dataset_utils.inject_outliers (utils/dataset_utils.py:436-461) on the device: a new SceneData
    whose measurements carry the injected outliers, or None when outlier sampling failed."""
    assert 0 < outlier_injection_rate < 1
    M = _dense_M(scene_data)
    inj = OutlierInjector(M, outlier_injection_rate, rng=rng, log=log)
    if inj.select_outliers(n_tries=5) is None:
        return None
    M_new = inj.inject_outliers(z=z, generator=generator)
    dev = M.device
    Ns = scene_data.Ns.to(dev, torch.float32).contiguous()
    y = scene_data.y.to(dev) if scene_data.y is not None else None
    out = scene_from_dense_device(M_new, Ns, y, scene_data.scene_name,
                                  calibrated=getattr(scene_data, "calibrated", True), max_piece=max_piece)
    out.outliers_mask = inj.outliers_mask
    # the reference passes these through to the rebuilt SceneData (dataset_utils.py:451-459); outlier
    # injection moves measurements of existing observations only, so the depth targets still apply
    for k in ("store_depth_targets", "depths"):
        if getattr(scene_data, k, None) is not None:
            setattr(out, k, getattr(scene_data, k))
    return out
