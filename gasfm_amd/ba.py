"""Bundle adjustment on the device: ``euc_ba`` / ``proj_ba`` of
code/utils/ba_functions.py:6-137 with the Ceres solve (ceres_utils.py:127-245,
bundle_adjustment/custom_cpp_cost_functions.cpp:56-222) replaced by an fp64 trust-region
Levenberg-Marquardt whose passes are HIP kernels (csrc/bundle_adjust.hip).

The problem is the reference's: per observation (camera c, point p) a 2-vector residual,
Euclidean (angle-axis + translation deltas on top of the initial camera, fixed K) or projective
(12 deltas of the column-major 3x4 P), point deltas on X (W = 1), HuberLoss(0.1), Ceres' defaults
for everything the reference leaves unset, ``function_tolerance = 1e-4``,
``max_num_iterations = 100``, DENSE_SCHUR.  The solver restates Ceres 2.1's
TrustRegionMinimizer + LevenbergMarquardtStrategy (oracle/ba.py lists the rules); each iteration:

  gasfm_ba_eval      residuals, corrected + Jacobi-scaled Jacobians, cost        (edges)
  gasfm_ba_normals   camera blocks U, gc (wave per camera), point blocks V, gp  (thread per point)
  gasfm_ba_damp      + LM diagonal / radius, V^-1
  gasfm_ba_schur     Y = W V^-1 per edge, rhs, the reduced camera matrix S by camera-pair
                     blocks over pair lists sorted once per problem (deterministic)
  rocSOLVER          Cholesky of S (torch.linalg.cholesky_ex) and the camera step
  gasfm_ba_backsub   point step (thread per point)
  gasfm_ba_model     model cost change (edges);  gasfm_ba_eval at the candidate (cost only)

The host keeps the scalar trust-region logic (a few 8-byte reads per iteration).  DLT
triangulation (``repeat`` / ``triangulation``) is gasfm_ba_dlt, camera matrices / normalisation /
reprojection errors are small fp64 torch ops on the device.
"""
import math

import numpy as np
import torch

from . import _native

F64 = torch.float64


# ------------------------------------------------------------------ native wrappers
def _p(t):
    return _native._p(t)


def _st(t):
    return _native._stream(t)


def _check(st, what):
    _native.check(st, what)


def _dev64(t, dev):
    return torch.as_tensor(t, dtype=F64).to(dev).contiguous()


# ------------------------------------------------------------------ rotations (cv2.Rodrigues semantics)
def rodrigues_to_matrix(r):
    """Rotation vectors [.., 3] -> matrices [.., 3, 3] (float64 torch)."""
    th = torch.linalg.norm(r, dim=-1, keepdim=True)
    small = th < 1e-300
    k = r / torch.where(small, torch.ones_like(th), th)
    z = torch.zeros_like(k[..., 0])
    Kx = torch.stack([z, -k[..., 2], k[..., 1], k[..., 2], z, -k[..., 0], -k[..., 1], k[..., 0], z], -1)
    Kx = Kx.reshape(r.shape[:-1] + (3, 3))
    s, c = torch.sin(th)[..., None], torch.cos(th)[..., None]
    I = torch.eye(3, dtype=r.dtype, device=r.device).expand(Kx.shape)
    return I + s * Kx + (1 - c) * (Kx @ Kx)


def matrix_to_rodrigues(R):
    """Log map of rotation matrices [.., 3, 3] -> rotation vectors [.., 3] (float64 numpy or torch)."""
    Rn = torch.as_tensor(R, dtype=F64)
    tr = Rn[..., 0, 0] + Rn[..., 1, 1] + Rn[..., 2, 2]
    th = torch.arccos(torch.clamp((tr - 1) / 2, -1.0, 1.0))
    v = torch.stack([Rn[..., 2, 1] - Rn[..., 1, 2], Rn[..., 0, 2] - Rn[..., 2, 0], Rn[..., 1, 0] - Rn[..., 0, 1]], -1)
    sin_th = torch.sin(th)
    out = torch.where((th < 1e-7)[..., None], v / 2, v * (th / (2 * torch.where(sin_th == 0, torch.ones_like(th),
                                                                                   sin_th)))[..., None])
    near_pi = (math.pi - th) < 1e-5
    if bool(near_pi.any()):  # axis from the symmetric part
        idx = torch.nonzero(near_pi.reshape(-1)).view(-1)
        Rf, vf, tf = Rn.reshape(-1, 3, 3), v.reshape(-1, 3), th.reshape(-1)
        of = out.reshape(-1, 3).clone()
        for i in idx.tolist():
            B = (Rf[i] + torch.eye(3, dtype=F64, device=Rf.device)) / 2
            j = int(torch.argmax(torch.diagonal(B)))
            k = B[:, j] / torch.sqrt(B[j, j])
            if float(k @ vf[i]) < 0:
                k = -k
            of[i] = k * tf[i]
        out = of.reshape(out.shape)
    return out


# ------------------------------------------------------------------ the problem
class BAProblem:
    """One Ceres problem: edges (cidx, pidx) camera-major with observations obs [E, 2], initial
    cameras cam0 [m, 6] (+ K [m, 5], Euclidean) or [m, 12] (projective), initial points X0 [n, 3];
    the unknowns are deltas (the reference's Psu / Xsu)."""

    def __init__(self, kind, cam0, X0, cidx, pidx, obs, K=None):
        assert kind in ("euc", "proj")
        self.kind = kind
        self.CP = 6 if kind == "euc" else 12
        dev = cam0.device
        if dev.type != "cuda":
            raise TypeError("BAProblem: tensors must be on the GPU (no CPU fallback)")
        self.dev = dev
        self.cam0 = cam0.to(F64).contiguous()
        self.X0 = X0.to(F64).contiguous()
        self.K = K.to(F64).contiguous() if K is not None else None
        self.m, self.n = self.cam0.shape[0], self.X0.shape[0]
        cidx = cidx.to(torch.int64)
        pidx = pidx.to(torch.int64)
        E = int(cidx.shape[0])
        if E == 0:
            raise ValueError("BAProblem: no observations")
        key = cidx * self.n + pidx
        if E > 1 and not bool((key[1:] > key[:-1]).all()):
            raise ValueError("BAProblem: observations must be unique and camera-major sorted")
        self.E = E
        self.cidx = cidx.to(torch.int32).contiguous()
        self.pidx = pidx.to(torch.int32).contiguous()
        self.obs = obs.to(F64).contiguous()
        i32 = dict(dtype=torch.int32, device=dev)
        self.cam_ptr = torch.zeros(self.m + 1, **i32)
        self.cam_ptr[1:] = torch.cumsum(torch.bincount(cidx, minlength=self.m), 0).to(torch.int32)
        cnt_p = torch.bincount(pidx, minlength=self.n)
        self.pt_ptr = torch.zeros(self.n + 1, **i32)
        self.pt_ptr[1:] = torch.cumsum(cnt_p, 0).to(torch.int32)
        perm = torch.argsort(pidx, stable=True)  # cameras ascending inside a point
        self.perm = perm.to(torch.int32).contiguous()
        self._build_pairs(perm, cidx, cnt_p)
        f = dict(dtype=F64, device=dev)
        CP = self.CP
        self.fres = torch.empty((E, 2), **f)
        self.Jc = torch.empty((E, 2, CP), **f)
        self.Jp = torch.empty((E, 2, 3), **f)
        self.U = torch.empty((self.m, CP, CP), **f)
        self.gc = torch.empty((self.m, CP), **f)
        self.V = torch.empty((self.n, 3, 3), **f)
        self.gp = torch.empty((self.n, 3), **f)
        self.Ud = torch.empty_like(self.U)
        self.Vinv = torch.empty_like(self.V)
        self.Y = torch.empty((E, CP, 3), **f)
        self.S = torch.empty((self.m * CP, self.m * CP), **f)
        self.rhs = torch.empty(self.m * CP, **f)
        self.dp = torch.empty((self.n, 3), **f)
        self.part = torch.empty(int(_native.lib().gasfm_ba_partials(E)), **f)
        self.scalar = torch.empty(1, **f)
        self.bad = torch.zeros(1, **i32)
        self.sc = None
        self.sp = None

    def _build_pairs(self, perm, cidx, cnt_p):
        """Edge pairs (e1 on camera a, e2 on camera b >= a) sharing a point, sorted by (a, b) once;
        camera-pair blocks with their pair ranges."""
        E, dev = self.E, self.dev
        slot_pt = torch.repeat_interleave(torch.arange(self.n, device=dev), cnt_p, output_size=E)
        end = self.pt_ptr[1:].to(torch.int64)[slot_pt]
        cnt = end - torch.arange(E, device=dev)
        P = int(cnt.sum())
        s1 = torch.repeat_interleave(torch.arange(E, device=dev), cnt, output_size=P)
        first = torch.cumsum(cnt, 0) - cnt
        s2 = s1 + (torch.arange(P, device=dev) - first[s1])
        e1, e2 = perm[s1], perm[s2]
        key = cidx[e1] * self.m + cidx[e2]
        order = torch.argsort(key, stable=True)
        key = key[order]
        self.pe1 = e1[order].to(torch.int32).contiguous()
        self.pe2 = e2[order].to(torch.int32).contiguous()
        ukey, counts = torch.unique_consecutive(key, return_counts=True)
        self.nblk = int(ukey.shape[0])
        self.blk_ptr = torch.zeros(self.nblk + 1, dtype=torch.int32, device=dev)
        self.blk_ptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        self.blk_ab = torch.stack([ukey // self.m, ukey % self.m], 1).to(torch.int32).contiguous()
        self.n_pairs = P

    # ---- passes
    def _sum(self):
        L = _native.lib()
        _check(L.gasfm_ba_sum(_p(self.part), self.part.shape[0], _p(self.scalar), _st(self.part)), "gasfm_ba_sum")
        return float(self.scalar.item())

    def evaluate(self, dcam, dX, jac):
        """Cost at (cam0 + dcam, X0 + dX); with jac, fills fres / Jc / Jp (scaled by sc / sp)."""
        L = _native.lib()
        _check(L.gasfm_ba_eval(self.CP, _p(self.cam0), _p(self.K), _p(self.X0), _p(dcam), _p(dX), _p(self.cidx),
                               _p(self.pidx), _p(self.obs), self.E, _p(self.sc), _p(self.sp), int(jac),
                               _p(self.fres), _p(self.Jc), _p(self.Jp), _p(self.part), _st(self.obs)), "gasfm_ba_eval")
        return self._sum()

    def normals(self):
        L = _native.lib()
        _check(L.gasfm_ba_normals(self.CP, self.m, self.n, _p(self.cam_ptr), _p(self.pt_ptr), _p(self.perm),
                                  _p(self.fres), _p(self.Jc), _p(self.Jp), _p(self.U), _p(self.gc), _p(self.V),
                                  _p(self.gp), _st(self.obs)), "gasfm_ba_normals")

    def step(self, radius):
        """LM step in scaled coordinates (dc [m, CP], dp [n, 3]) or None when a factorisation fails."""
        L = _native.lib()
        st = _st(self.obs)
        self.bad.zero_()
        _check(L.gasfm_ba_damp(self.CP, self.m, self.n, _p(self.U), _p(self.V), float(radius), _p(self.Ud),
                               _p(self.Vinv), _p(self.bad), st), "gasfm_ba_damp")
        _check(L.gasfm_ba_schur(self.CP, self.m, _p(self.cam_ptr), _p(self.cidx), _p(self.pidx), self.E, _p(self.Jc),
                                _p(self.Jp), _p(self.Vinv), _p(self.gc), _p(self.gp), _p(self.Ud), _p(self.blk_ptr),
                                _p(self.blk_ab), self.nblk, _p(self.pe1), _p(self.pe2), _p(self.Y), _p(self.S),
                                _p(self.rhs), st), "gasfm_ba_schur")
        Lc, info = torch.linalg.cholesky_ex(self.S)
        if int(info.item()) != 0 or int(self.bad.item()) != 0:
            return None
        dc = torch.cholesky_solve(self.rhs[:, None], Lc)[:, 0].reshape(self.m, self.CP).contiguous()
        _check(L.gasfm_ba_backsub(self.CP, self.n, _p(self.pt_ptr), _p(self.perm), _p(self.cidx), _p(self.Jc),
                                  _p(self.Jp), _p(self.Vinv), _p(self.gp), _p(dc), _p(self.dp), st), "gasfm_ba_backsub")
        return dc, self.dp.clone()

    def model_change(self, dc, dp):
        L = _native.lib()
        _check(L.gasfm_ba_model(self.CP, _p(self.cidx), _p(self.pidx), self.E, _p(self.Jc), _p(self.Jp),
                                _p(self.fres), _p(dc), _p(dp), _p(self.part), _st(self.obs)), "gasfm_ba_model")
        return self._sum()

    # ---- the minimizer
    def solve(self, max_iter=100, ftol=1e-4, gtol=1e-10, ptol=1e-8, log=None):
        """Ceres trust-region LM (oracle/ba.py) -> (dcam [m, CP], dX [n, 3], summary)."""
        f = dict(dtype=F64, device=self.dev)
        dcam = torch.zeros((self.m, self.CP), **f)
        dX = torch.zeros((self.n, 3), **f)
        self.sc = self.sp = None
        self.evaluate(dcam, dX, True)
        self.normals()
        # Jacobi scaling fixed at iteration 0: 1 / (1 + |column|)
        self.sc = (1.0 / (1.0 + torch.sqrt(torch.diagonal(self.U, dim1=1, dim2=2)))).contiguous()
        self.sp = (1.0 / (1.0 + torch.sqrt(torch.diagonal(self.V, dim1=1, dim2=2)))).contiguous()
        cost = self.evaluate(dcam, dX, True)
        self.normals()
        summ = {"initial_cost": cost, "iterations": 0, "successful": 0, "termination": "NO_CONVERGENCE",
                "costs": [cost]}

        def grad_max():
            return float(torch.maximum((self.gc / self.sc).abs().max(), (self.gp / self.sp).abs().max()).item())

        if grad_max() <= gtol:
            summ["termination"] = "CONVERGENCE"
            summ["final_cost"] = cost
            return dcam, dX, summ
        radius, dec = 1e4, 2.0
        for it in range(1, max_iter + 1):
            summ["iterations"] = it
            st = self.step(radius)
            rho = -math.inf
            if st is not None:
                dc, dp = st
                model = self.model_change(dc, dp)
                delta_c, delta_p = dc * self.sc, dp * self.sp
                step_norm = math.sqrt(float((delta_c * delta_c).sum() + (delta_p * delta_p).sum()))
                x_norm = math.sqrt(float((dcam * dcam).sum() + (dX * dX).sum()))
                if step_norm <= ptol * (x_norm + ptol):
                    summ["termination"] = "CONVERGENCE"
                    break
                cand_c, cand_p = dcam + delta_c, dX + delta_p
                cand = self.evaluate(cand_c, cand_p, False)
                change = cost - cand
                if abs(change) <= ftol * cost:
                    summ["termination"] = "CONVERGENCE"
                    break
                if model > 0:
                    rho = change / model
            if rho > 1e-3:
                dcam, dX = cand_c, cand_p
                cost = self.evaluate(dcam, dX, True)
                self.normals()
                summ["successful"] += 1
                summ["costs"].append(cost)
                radius = min(radius / max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3), 1e16)
                dec = 2.0
                if grad_max() <= gtol:
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
        return dcam, dX, summ


# ------------------------------------------------------------------ geometry on the device
def valid_points(xs):
    """get_M_valid_points on [m, n, 2] (dataset_utils.py:86-113): nonzero and >= 2 views."""
    v = xs.abs().sum(dim=2) != 0
    v[:, v.sum(dim=0) < 2] = False
    return v


def camera_matrices(Rs, ts, Ks):
    """K R^T [I | -t] (geo_utils.get_camera_matrix, :294-315)."""
    Rt = Rs.transpose(1, 2)
    return Ks @ torch.cat([Rt, -(Rt @ ts[:, :, None])], dim=2)


def normalized_observations(Ns, cidx, obs):
    """(N_c [x, y, 1]^T) / z per edge (geo_utils.normalize_points_cams, :536-560)."""
    h = torch.cat([obs, torch.ones_like(obs[:, :1])], 1)
    q = (Ns[cidx.long()] @ h[:, :, None])[:, :, 0]
    z = torch.where(q[:, 2] == 0, torch.ones_like(q[:, 2]), q[:, 2])
    return (q[:, :2] / z[:, None]).contiguous()


class _Edges:
    def __init__(self, xs):
        vis = valid_points(xs)
        c, p = torch.nonzero(vis, as_tuple=True)  # camera-major (the reference's np.where order)
        self.vis, self.cidx, self.pidx = vis, c, p
        self.obs = xs[c, p].contiguous()
        self.m, self.n = xs.shape[0], xs.shape[1]
        cnt = torch.bincount(p, minlength=self.n)
        self.pt_ptr = torch.zeros(self.n + 1, dtype=torch.int32, device=xs.device)
        self.pt_ptr[1:] = torch.cumsum(cnt, 0).to(torch.int32)
        self.perm = torch.argsort(p, stable=True).to(torch.int32).contiguous()
        self.c32 = c.to(torch.int32).contiguous()

    def repro(self, Ps, Xs):
        """nanmean of reprojection_error_with_points (geo_utils.py:371-391) over the visible entries."""
        X4 = torch.cat([Xs[:, :3], torch.ones_like(Xs[:, :1])], 1) if Xs.shape[1] == 3 else Xs
        q = (Ps[self.cidx] @ X4[self.pidx][:, :, None])[:, :, 0]
        err = torch.linalg.norm(self.obs - q[:, :2] / q[:, 2:3], dim=1)
        ok = ~torch.isnan(err)
        return float(err[ok].mean().item()) if bool(ok.any()) else float("nan")

    def dlt(self, Ps, Ns):
        """dlt_triangulation on the normalised cameras / points (gasfm_ba_dlt): [n, 4]."""
        nP = (Ns @ Ps).contiguous()
        nx = normalized_observations(Ns, self.cidx, self.obs)
        X = torch.empty((self.n, 4), dtype=F64, device=Ps.device)
        _check(_native.lib().gasfm_ba_dlt(self.n, _p(self.pt_ptr), _p(self.perm), _p(self.c32), _p(nP), _p(nx), _p(X),
                                          _st(X)), "gasfm_ba_dlt")
        return X


def _euc_params(Rs, ts, Ks):
    """order_cam_param_for_c (ceres_utils.py:11-29): (aa, t) and K (K00 K01 K02 K11 K12)."""
    Rt = Rs.transpose(1, 2)
    cam = torch.cat([matrix_to_rodrigues(Rt).to(Rs.device), -(Rt @ ts[:, :, None])[:, :, 0]], 1)
    K = torch.stack([Ks[:, 0, 0], Ks[:, 0, 1], Ks[:, 0, 2], Ks[:, 1, 1], Ks[:, 1, 2]], 1)
    return cam.contiguous(), K.contiguous()


def _euc_from_params(cam, Ks):
    """reorder_from_c_to_py (ceres_utils.py:32-48)."""
    Rs = rodrigues_to_matrix(cam[:, :3]).transpose(1, 2)
    ts = -(Rs @ cam[:, 3:6, None])[:, :, 0]
    return Rs, ts, camera_matrices(Rs, ts, Ks)


def _report(print_out, tag, s):
    if print_out:
        print(f"[gasfm ba] {tag}: {s['termination']} after {s['iterations']} iterations "
              f"({s['successful']} successful), cost {s['initial_cost']:.6e} -> {s['final_cost']:.6e}")


def run_euclidean(Xs, ed, Rs, ts, Ks, print_out=False, tag="ba", **kw):
    cam0, K = _euc_params(Rs, ts, Ks)
    prob = BAProblem("euc", cam0, Xs[:, :3], ed.cidx, ed.pidx, ed.obs, K)
    dc, dX, summ = prob.solve(**kw)
    _report(print_out, tag, summ)
    Rn, tn, Pn = _euc_from_params(cam0 + dc, Ks)
    return Rn, tn, Pn, Xs[:, :3] + dX, summ["termination"] != "FAILURE", summ


def _as_dev(x, dev):
    return None if x is None else torch.as_tensor(np.asarray(x) if not torch.is_tensor(x) else x).to(dev, F64)


def _out(res, numpy_out):
    if not numpy_out:
        return res
    return {k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in res.items()}


def euc_ba(xs, Rs, ts, Ks, Xs_our=None, Ps=None, Ns=None, repeat=True, triangulation=False, return_repro=True,
           print_out=True, device=None, **solver):
    """ba_functions.euc_ba (code/utils/ba_functions.py:6-72) on the GPU.  Same arguments and
    results (numpy in -> numpy out; CUDA tensors in -> tensors out): Rs, ts, Ps, Xs [n, 4] and,
    with return_repro, repro_before / _middle / _middle_triangulated / _after."""
    numpy_out = not torch.is_tensor(xs)
    dev = device or (xs.device if torch.is_tensor(xs) and xs.is_cuda else torch.device("cuda", 0))
    xs, Rs, ts, Ks = (_as_dev(a, dev) for a in (xs, Rs, ts, Ks))
    Ps, Ns, Xs_our = _as_dev(Ps, dev), _as_dev(Ns, dev), _as_dev(Xs_our, dev)
    res = {}
    ed = _Edges(xs)
    if Ps is None:
        Ps = camera_matrices(Rs, ts, Ks)
    if triangulation:
        if Ns is None:
            Ns = torch.linalg.inv(Ks)
        Xs = ed.dlt(Ps, Ns)
    else:
        Xs = Xs_our
    if return_repro:
        res["repro_before"] = ed.repro(Ps, Xs)
    Rn, tn, Pn, Xn, ok, s1 = run_euclidean(Xs, ed, Rs, ts, Ks, print_out, "ba 1", **solver)
    res["converged1"], res["summary1"] = ok, s1
    if repeat:
        if return_repro:
            res["repro_middle"] = ed.repro(Pn, Xn)
        if Ns is None:
            Ns = torch.linalg.inv(Ks)
        Xn = ed.dlt(Pn, Ns)
        if return_repro:
            res["repro_middle_triangulated"] = ed.repro(Pn, Xn)
        Rn, tn, Pn, Xn, ok, s2 = run_euclidean(Xn, ed, Rn, tn, Ks, print_out, "ba 2", **solver)
        res["converged2"], res["summary2"] = ok, s2
    if return_repro:
        res["repro_after"] = ed.repro(Pn, Xn)
    res["Rs"], res["ts"], res["Ps"] = Rn, tn, Pn
    res["Xs"] = torch.cat([Xn[:, :3], torch.ones_like(Xn[:, :1])], 1)
    return _out(res, numpy_out)


def run_projective(Ps, Xs, ed, print_out=False, tag="ba", **kw):
    m = Ps.shape[0]
    P0 = Ps.transpose(1, 2).reshape(m, 12).contiguous()  # column-major 3x4 (ceres_utils.py:219-220)
    prob = BAProblem("proj", P0, Xs[:, :3], ed.cidx, ed.pidx, ed.obs)
    dc, dX, summ = prob.solve(**kw)
    _report(print_out, tag, summ)
    return (P0 + dc).reshape(m, 4, 3).transpose(1, 2), Xs[:, :3] + dX, summ["termination"] != "FAILURE", summ


def proj_ba(Ps, xs, Xs_our=None, Ns=None, repeat=True, triangulation=False, return_repro=True, normalize_in_tri=True,
            print_out=True, device=None, **solver):
    """ba_functions.proj_ba (code/utils/ba_functions.py:75-137) on the GPU; Ns is required when
    triangulating with normalisation (the reference then derives it from the points otherwise)."""
    numpy_out = not torch.is_tensor(xs)
    dev = device or (xs.device if torch.is_tensor(xs) and xs.is_cuda else torch.device("cuda", 0))
    xs, Ps, Ns, Xs_our = (_as_dev(a, dev) for a in (xs, Ps, Ns, Xs_our))
    if (triangulation or repeat) and normalize_in_tri and Ns is None:
        raise ValueError("proj_ba: pass Ns (normalisation matrices) for the normalised triangulation")
    res = {}
    ed = _Edges(xs)
    eye = torch.eye(3, dtype=F64, device=dev).expand(Ps.shape[0], 3, 3)
    Nt = Ns if normalize_in_tri else eye
    Xs = ed.dlt(Ps, Nt) if triangulation else Xs_our
    if return_repro:
        res["repro_before"] = ed.repro(Ps, Xs)
    Pn, Xn, ok, s1 = run_projective(Ps, Xs, ed, print_out, "ba 1", **solver)
    res["converged1"], res["summary1"] = ok, s1
    if repeat:
        if return_repro:
            res["repro_middle"] = ed.repro(Pn, Xn)
        Xn = ed.dlt(Pn, Nt)
        if return_repro:
            res["repro_middle_triangulated"] = ed.repro(Pn, Xn)
        Pn, Xn, ok, s2 = run_projective(Pn, Xn, ed, print_out, "ba 2", **solver)
        res["converged2"], res["summary2"] = ok, s2
    if return_repro:
        res["repro_after"] = ed.repro(Pn, Xn)
    res["Ps"] = Pn
    res["Xs"] = torch.cat([Xn[:, :3], torch.ones_like(Xn[:, :1])], 1)
    return _out(res, numpy_out)
