"""CPU restatement of the reference's bundle adjustment (TEST INFRASTRUCTURE ONLY).

Only tests/ may import this module, as the checker of gasfm_amd.ba (the device path).

The reference refines a prediction with Ceres (code/utils/ba_functions.py:6-137,
code/utils/ceres_utils.py:127-245, bundle_adjustment/custom_cpp_cost_functions.cpp:56-222):

  residual (Euclidean, eucReprojectionError :105-155), camera block P = (angle-axis 3, t 3) as
      DELTAS added to the initial values (Porig, Xorig):
      Xc = AngleAxisRotatePoint(aa0 + daa, X0 + dX) + (t0 + dt)
      r  = ((K00 Xc0 + K01 Xc1 + K02 Xc2) / Xc2 - x,  (K11 Xc1 + K12 Xc2) / Xc2 - y)
      aa0 = Rodrigues(R^T), t0 = -R^T t, K fixed (order_cam_param_for_c, ceres_utils.py:11-29)
  residual (projective, projReprojectionError :56-102): P (12, column-major, deltas) and
      X (3, W = 1):  r = (P X)_xy / (P X)_z - x
  loss HuberLoss(0.1); DENSE_SCHUR; function_tolerance 1e-4; max_num_iterations 100.

Ceres 2.1 is absent (no headers, no library): the solver below restates its documented
trust-region Levenberg-Marquardt with the defaults the reference leaves untouched --
Jacobi column scaling 1 / (1 + |J_col|) fixed at iteration 0, LM diagonal diag(J^T J) clamped
to [1e-6, 1e32] and divided by the radius (initial 1e4, max 1e16; on success
radius / max(1/3, 1 - (2 rho - 1)^3), on failure radius / 2, 4, 8, ...), a step succeeds when
its relative decrease exceeds 1e-3, stop when |cost change| <= 1e-4 cost (the candidate is not
taken), |step| <= 1e-8 (|x| + 1e-8) or max |gradient| <= 1e-10; the Huber loss enters through
Ceres' corrector, which for Huber scales residual and Jacobian by sqrt(rho'(s)).  Jacobians by
complex-step differentiation of the residual (exact to rounding, independent of the device's
dual numbers).  DLT triangulation, camera matrices, normalisation and reprojection errors restate
code/utils/geo_utils.py:294-315, 371-391, 536-560, 611-656 and are pinned to the reference's own
outputs (tests/golden/ba.npz, make_golden_ba.py); the LM trajectory itself is "parity unpinned"
against Ceres (absent), and pinned by known answers (noise-free scenes converge to zero error).
"""
import numpy as np

HUBER_A = 0.1
EPS = np.finfo(np.float64).eps


# ------------------------------------------------------------------ geometry (geo_utils.py restated)
def valid_points(xs):
    """get_M_valid_points on [m, n, 2]: nonzero measurement and >= 2 views per point."""
    v = np.abs(xs).sum(axis=2) != 0
    v[:, v.sum(axis=0) < 2] = False
    return v


def camera_matrix(R, t, K):
    return K @ R.T @ np.concatenate((np.eye(3), -t.reshape(3, 1)), axis=1)


def camera_matrices(Rs, ts, Ks):
    return np.stack([camera_matrix(r, t, k) for r, t, k in zip(Rs, ts, Ks)])


def reprojection_errors(Ps, Xs, xs, visible=None):
    m, n, _ = xs.shape
    X4 = np.concatenate([Xs, np.ones([n, 1])], axis=1) if Xs.shape[1] == 3 else Xs
    if visible is None:
        visible = valid_points(xs)
    proj = (Ps @ X4.T).swapaxes(1, 2)
    vi = np.nonzero(visible)
    proj[vi[0], vi[1], :] = proj[vi[0], vi[1], :] / proj[vi[0], vi[1], -1][:, None]
    err = np.linalg.norm(xs[:, :, :2] - proj[:, :, :2], axis=2)
    err[~visible] = np.nan
    return err


def normalize_points_cams(Ps, xs, Ns):
    m, n, d = xs.shape
    xs3 = np.concatenate([xs, np.ones([m, n, 1])], axis=2) if d == 2 else xs
    nP, nx = np.zeros_like(Ps), np.zeros_like(xs)
    for i in range(m):
        nP[i] = Ns[i] @ Ps[i]
        q = (Ns[i] @ xs3[i].T).T
        q[q[:, -1] == 0, -1] = 1
        q = q / q[:, -1].reshape([-1, 1])
        nx[i] = q[:, :2] if d == 2 else q
    return nP, nx


def dlt_triangulation(Ps, xs, visible):
    """[n, 4] with X[3] = 1 (NaN for points in < 2 views): the null vector of the
    [3k x (k + 4)] system P_j X - lambda_j x_j = 0, by SVD as the reference."""
    m, n, _ = xs.shape
    X = np.zeros([n, 4])
    for i in range(n):
        cams = np.where(visible[:, i])[0]
        k = len(cams)
        if k < 2:
            X[i] = np.nan
            continue
        A = np.zeros([3 * k, k + 4])
        for j, c in enumerate(cams):
            A[3 * j:3 * j + 3, :4] = Ps[c]
            A[3 * j:3 * j + 2, 4 + j] = -xs[c, i, :2]
            A[3 * j + 2, 4 + j] = -1
        _, _, Vh = np.linalg.svd(A)
        v = Vh[-1, :4]
        X[i] = v / v[-1]
    return X


# ------------------------------------------------------------------ rotations
def rodrigues_to_matrix(r):
    th = np.linalg.norm(r)
    if th < 1e-300:
        return np.eye(3)
    k = r / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * (Kx @ Kx)


def matrix_to_rodrigues(R):
    """log map of a rotation matrix (the value cv2.Rodrigues returns for a rotation)."""
    c = np.clip((np.trace(R) - 1) / 2, -1.0, 1.0)
    th = np.arccos(c)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    if th < 1e-7:
        return v / 2
    if np.pi - th < 1e-5:  # near pi: axis from the symmetric part
        B = (R + np.eye(3)) / 2
        k = np.sqrt(np.clip(np.diag(B), 0, None))
        i = int(np.argmax(k))
        k = B[:, i] / np.sqrt(B[i, i])
        if np.dot(k, v) < 0:
            k = -k
        return k * th
    return v * (th / (2 * np.sin(th)))


def angle_axis_rotate_point(aa, p):
    """ceres::AngleAxisRotatePoint (rotation.h), elementwise over leading dims; complex-safe."""
    t2 = (aa * aa).sum(-1)
    big = np.real(t2) > EPS
    th = np.sqrt(np.where(big, t2, 1.0))
    c, s = np.cos(th), np.sin(th)
    w = aa / th[..., None]
    wxp = np.cross(w, p)
    tmp = (w * p).sum(-1) * (1 - c)
    r_big = p * c[..., None] + wxp * s[..., None] + w * tmp[..., None]
    r_small = p + np.cross(aa, p)
    return np.where(big[..., None], r_big, r_small)


# ------------------------------------------------------------------ residuals
def euc_residual(cam, X, K, obs):
    """cam [.., 6] (aa, t), X [.., 3], K [.., 5] = (K00, K01, K02, K11, K12), obs [.., 2]."""
    Xc = angle_axis_rotate_point(cam[..., :3], X) + cam[..., 3:6]
    px = (Xc[..., 0] * K[..., 0] + Xc[..., 1] * K[..., 1] + Xc[..., 2] * K[..., 2]) / Xc[..., 2]
    py = (Xc[..., 1] * K[..., 3] + Xc[..., 2] * K[..., 4]) / Xc[..., 2]
    return np.stack([px - obs[..., 0], py - obs[..., 1]], -1)


def proj_residual(P, X, obs):
    """P [.., 12] column-major 3x4 (Ps.reshape(-1, 12, order="F")), X [.., 3] (W = 1)."""
    q = [P[..., r] * X[..., 0] + P[..., 3 + r] * X[..., 1] + P[..., 6 + r] * X[..., 2] + P[..., 9 + r] for r in range(3)]
    return np.stack([q[0] / q[2] - obs[..., 0], q[1] / q[2] - obs[..., 1]], -1)


def huber(s, a=HUBER_A):
    """ceres::HuberLoss::Evaluate: (rho, rho')."""
    b = a * a
    r = np.sqrt(np.maximum(s, 0))
    big = s > b
    rho = np.where(big, 2 * a * r - b, s)
    d1 = np.where(big, np.maximum(np.finfo(np.float64).tiny, a / np.where(big, r, 1.0)), 1.0)
    return rho, d1


class Problem:
    """Edges (cam, pt, obs) with the initial camera / point values (the Ceres Porig / Xorig)."""

    def __init__(self, kind, cam0, X0, cidx, pidx, obs, K=None):
        self.kind = kind
        self.cam0 = np.asarray(cam0, np.float64)
        self.X0 = np.asarray(X0, np.float64)
        self.cidx = np.asarray(cidx, np.int64)
        self.pidx = np.asarray(pidx, np.int64)
        self.obs = np.asarray(obs, np.float64)
        self.K = None if K is None else np.asarray(K, np.float64)
        self.m, self.n = self.cam0.shape[0], self.X0.shape[0]
        self.CP = 6 if kind == "euc" else 12
        self.N = self.m * self.CP + 3 * self.n

    def split(self, x):
        return x[:self.m * self.CP].reshape(self.m, self.CP), x[self.m * self.CP:].reshape(self.n, 3)

    def residuals(self, x):
        dc, dX = self.split(x)
        c = self.cam0 + dc
        X = self.X0 + dX
        if self.kind == "euc":
            return euc_residual(c[self.cidx], X[self.pidx], self.K[self.cidx], self.obs)
        return proj_residual(c[self.cidx], X[self.pidx], self.obs)

    def evaluate(self, x, jac=True):
        """cost, corrected residuals [E, 2] and corrected Jacobian [2E, N] (dense)."""
        r = self.residuals(x)
        s = (r * r).sum(-1)
        rho, d1 = huber(s)
        cost = 0.5 * rho.sum()
        w = np.sqrt(d1)
        f = (r * w[:, None]).reshape(-1)
        if not jac:
            return cost, f, None
        E = self.cidx.shape[0]
        J = np.zeros((2 * E, self.N))
        h = 1e-30
        dc0, dX0 = self.split(x)
        c = self.cam0 + dc0
        X = self.X0 + dX0
        ce, Xe = c[self.cidx].astype(np.complex128), X[self.pidx].astype(np.complex128)
        for k in range(self.CP + 3):
            cc, XX = ce.copy(), Xe.copy()
            if k < self.CP:
                cc[:, k] += 1j * h
            else:
                XX[:, k - self.CP] += 1j * h
            if self.kind == "euc":
                rr = euc_residual(cc, XX, self.K[self.cidx], self.obs)
            else:
                rr = proj_residual(cc, XX, self.obs)
            d = (rr.imag / h) * w[:, None]
            col = (self.cidx * self.CP + k) if k < self.CP else (self.m * self.CP + self.pidx * 3 + (k - self.CP))
            J[2 * np.arange(E), col] = d[:, 0]
            J[2 * np.arange(E) + 1, col] = d[:, 1]
        return cost, f, J


def solve(prob, max_iter=100, ftol=1e-4, gtol=1e-10, ptol=1e-8, log=None):
    """Ceres trust-region LM (see module doc) -> (x, summary dict)."""
    x = np.zeros(prob.N)
    cost, f, J = prob.evaluate(x)
    scale = 1.0 / (1.0 + np.sqrt((J * J).sum(0)))
    g = J.T @ f
    summ = {"initial_cost": cost, "iterations": 0, "successful": 0, "termination": "NO_CONVERGENCE", "costs": [cost]}
    if np.abs(g).max(initial=0) <= gtol:
        summ["termination"] = "CONVERGENCE"
        summ["final_cost"] = cost
        return x, summ
    radius, dec, diag = 1e4, 2.0, None
    for it in range(1, max_iter + 1):
        summ["iterations"] = it
        Js = J * scale
        if diag is None:
            diag = np.clip((Js * Js).sum(0), 1e-6, 1e32)
        A = Js.T @ Js + np.diag(diag / radius)
        try:
            L = np.linalg.cholesky(A)
            step = -np.linalg.solve(L.T, np.linalg.solve(L, Js.T @ f))
            ok = True
        except np.linalg.LinAlgError:
            ok = False
        if ok:
            mr = Js @ step
            model_change = -mr @ (f + mr / 2)
            delta = step * scale
            if np.linalg.norm(delta) <= ptol * (np.linalg.norm(x) + ptol):
                summ["termination"] = "CONVERGENCE"
                break
            cand, _, _ = prob.evaluate(x + delta, jac=False)
            change = cost - cand
            if abs(change) <= ftol * cost:
                summ["termination"] = "CONVERGENCE"
                break
            rho = change / model_change if model_change > 0 else -np.inf
        else:
            rho = -np.inf
        if rho > 1e-3:
            x = x + delta
            cost, f, J = prob.evaluate(x)
            summ["successful"] += 1
            summ["costs"].append(cost)
            radius = min(radius / max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3), 1e16)
            dec, diag = 2.0, None
            g = J.T @ f
            if np.abs(g).max() <= gtol:
                summ["termination"] = "CONVERGENCE"
                break
        else:
            radius /= dec
            dec *= 2.0
            if radius < 1e-32:
                summ["termination"] = "FAILURE"
                break
        if log:
            log(it, cost, radius)
    summ["final_cost"] = cost
    return x, summ


# ------------------------------------------------------------------ euc_ba / proj_ba
def euc_camera_params(Rs, ts, Ks):
    """order_cam_param_for_c (ceres_utils.py:11-29): (aa, t, K00 K01 K02 K11 K12) per camera."""
    m = len(Rs)
    cam = np.zeros((m, 6))
    K = np.zeros((m, 5))
    for i in range(m):
        cam[i, :3] = matrix_to_rodrigues(Rs[i].T)
        cam[i, 3:6] = -Rs[i].T @ ts[i]
        K[i] = [Ks[i, 0, 0], Ks[i, 0, 1], Ks[i, 0, 2], Ks[i, 1, 1], Ks[i, 1, 2]]
    return cam, K


def euc_from_params(cam, Ks):
    """reorder_from_c_to_py (ceres_utils.py:32-48)."""
    m = cam.shape[0]
    Rs, ts = np.zeros((m, 3, 3)), np.zeros((m, 3))
    for i in range(m):
        Rs[i] = rodrigues_to_matrix(cam[i, :3]).T
        ts[i] = -Rs[i] @ cam[i, 3:6]
    return Rs, ts, camera_matrices(Rs, ts, Ks)


def run_euclidean(Xs, xs_vis, Rs, ts, Ks, cidx, pidx, **kw):
    cam0, K = euc_camera_params(Rs, ts, Ks)
    prob = Problem("euc", cam0, Xs[:, :3], cidx, pidx, xs_vis, K)
    x, summ = solve(prob, **kw)
    dc, dX = prob.split(x)
    Rn, tn, Pn = euc_from_params(cam0 + dc, Ks)
    return Rn, tn, Pn, Xs[:, :3] + dX, summ["termination"] != "FAILURE", summ


def euc_ba(xs, Rs, ts, Ks, Xs_our=None, Ps=None, Ns=None, repeat=True, triangulation=False, **kw):
    """ba_functions.euc_ba (:6-72) with the restated solver."""
    res = {}
    vis = valid_points(xs)
    cidx, pidx = np.where(vis)
    xs_vis = xs[vis]
    if Ps is None:
        Ps = camera_matrices(Rs, ts, Ks)
    if Ns is None:
        Ns = np.linalg.inv(Ks)
    if triangulation:
        nP, nx = normalize_points_cams(Ps, xs, Ns)
        Xs = dlt_triangulation(nP, nx, vis)
    else:
        Xs = Xs_our
    res["repro_before"] = np.nanmean(reprojection_errors(Ps, Xs, xs, vis))
    Rn, tn, Pn, Xn, ok, s1 = run_euclidean(Xs, xs_vis, Rs, ts, Ks, cidx, pidx, **kw)
    res["converged1"], res["summary1"] = ok, s1
    if repeat:
        res["repro_middle"] = np.nanmean(reprojection_errors(Pn, Xn, xs, vis))
        nP, nx = normalize_points_cams(Pn, xs, Ns)
        Xn = dlt_triangulation(nP, nx, vis)
        res["repro_middle_triangulated"] = np.nanmean(reprojection_errors(Pn, Xn, xs, vis))
        Rn, tn, Pn, Xn, ok, s2 = run_euclidean(Xn, xs_vis, Rn, tn, Ks, cidx, pidx, **kw)
        res["converged2"], res["summary2"] = ok, s2
    res["repro_after"] = np.nanmean(reprojection_errors(Pn, Xn, xs, vis))
    res["Rs"], res["ts"], res["Ps"] = Rn, tn, Pn
    res["Xs"] = np.concatenate([Xn, np.ones([Xn.shape[0], 1])], axis=1)
    return res


def run_projective(Ps, Xs, xs_vis, cidx, pidx, **kw):
    m = Ps.shape[0]
    P0 = Ps.reshape([-1, 12], order="F")
    prob = Problem("proj", P0, Xs[:, :3], cidx, pidx, xs_vis)
    x, summ = solve(prob, **kw)
    dc, dX = prob.split(x)
    return (P0 + dc).reshape([m, 3, 4], order="F"), Xs[:, :3] + dX, summ["termination"] != "FAILURE", summ


def proj_ba(Ps, xs, Xs_our=None, Ns=None, repeat=True, triangulation=False, **kw):
    """ba_functions.proj_ba (:75-137) with the restated solver (normalize_in_tri=True, Ns given)."""
    res = {}
    vis = valid_points(xs)
    cidx, pidx = np.where(vis)
    xs_vis = xs[vis]
    if triangulation:
        nP, nx = normalize_points_cams(Ps, xs, Ns)
        Xs = dlt_triangulation(nP, nx, vis)
    else:
        Xs = Xs_our
    res["repro_before"] = np.nanmean(reprojection_errors(Ps, Xs, xs, vis))
    Pn, Xn, ok, s1 = run_projective(Ps, Xs, xs_vis, cidx, pidx, **kw)
    res["converged1"], res["summary1"] = ok, s1
    if repeat:
        res["repro_middle"] = np.nanmean(reprojection_errors(Pn, Xn, xs, vis))
        nP, nx = normalize_points_cams(Pn, xs, Ns)
        Xn = dlt_triangulation(nP, nx, vis)
        res["repro_middle_triangulated"] = np.nanmean(reprojection_errors(Pn, Xn, xs, vis))
        Pn, Xn, ok, s2 = run_projective(Pn, Xn, xs_vis, cidx, pidx, **kw)
        res["converged2"], res["summary2"] = ok, s2
    res["repro_after"] = np.nanmean(reprojection_errors(Pn, Xn, xs, vis))
    res["Ps"] = Pn
    res["Xs"] = np.concatenate([Xn, np.ones([Xn.shape[0], 1])], axis=1)
    return res
