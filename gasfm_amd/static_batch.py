"""Shape-stable union batches: the config-3 / config-5 training step as ONE replayed hipGraph.

train.py (:60-152) samples a batch of scenes per step (10-20 views each, rotational augmentation,
config 5 also outlier injection), runs the model per scene, sums the ESFMLoss terms and steps Adam.
``batch.SceneBatch`` already runs the batch as one forward over the union graph, but every step has
new camera / point / edge counts, so the ~4,000 launches of forward + loss + backward are issued
from Python each time: the step is host-bound (``tools/train_step_bench.py``: ~35 ms eager against
~9.5 ms for the same launches replayed).  A replayed graph needs every launch parameter and every
buffer size fixed.  Here the union is padded to a BUCKET of fixed sizes with one extra pad scene --
a real, disjoint graph of the bucket's remaining cameras, points and edges -- so that every
quantity that sizes a launch is a function of the bucket alone:

  quantity                         real scenes                          pad scene (index B)
  -------------------------------  -----------------------------------  ------------------------------
  cameras / points / edges         concatenated (batch.SceneBatch)      M_cap - M / N_cap - N / E_cap - E
  camera plan (proj2view)          ceil(deg / 256) pieces per camera    the rest of the I_cap pieces,
                                   EVERY camera through partial slots   spread over the pad cameras
                                   + one combine entry per camera
                                   (I_cap items, M_cap combines)
  point plan (proj2scenepoint)     one item per point (deg <= 256)      one item per pad point
  view2global                      V2G_PIECES pieces per scene, every   all pad cameras valid
                                   scene split, one-level combine       (>= 8 edges each)
  scenepoint2global                S2G_PIECES pieces per scene, every   all pad points valid
                                   scene split, fixed two-level combine (2..256 edges each)

The pad scene's edges are cam-major and point-sorted at once (edge k joins the k-th entries of the
two degree expansions), its measurements are zero, and the loss gives it weight 0: its cameras' and
points' loss gradients are exact zeros (gasfm_esfm_seg_bwd), so it changes neither the real
scenes' forward (the scenes are disjoint in every aggregation) nor any parameter gradient.  The
real scenes see exactly the eager union's computation except that a one-piece camera goes through a
partial slot and a one-entry combine (the same merge arithmetic), the global graphs use other piece
lengths, and the loss sums per-scene partials in another order: fp32 summation-order differences
(tests/test_gpu_static_batch.py).

``StaticTrainer`` keeps one ``StaticBatch`` + ``graph_step.CapturedStep`` per bucket (all graphs in
one memory pool, replayed one at a time), fills the sampled batch into the bucket's static input
buffers with device copies (one host read of the batch statistics), replays, and leaves the
gradients in ``p.grad`` for the optimizer.  A batch takes the smallest existing bucket it fits
within the waste bound, else a new bucket is made and captured (a few eager warm-up passes on that
batch, whose gradients are the step's).  Batches the scheme cannot express (a camera without edges,
a point seen by > 256 views, a scene with < S2G_PIECES valid points) run eagerly through
batch.SceneBatch, counted in ``StaticTrainer.eager_steps``.
"""
import math
import time

import numpy as np
import torch

from . import _native
from .attention import DEFAULT_MAX_PIECE, AttnPlan
from .batch import _scene_arrays
from .graph_step import gc_paused
from .model import EdgeIndex
from .scene import MIN_N_POINTS_PER_VIEW, MIN_N_VIEWS_PER_POINT, AxialAggregationGraphWrapper, SparseMat

PIECE = DEFAULT_MAX_PIECE  # camera pieces: ceil(deg / PIECE) per real camera, as the eager plans
S2G_PIECES = 512  # pieces per scene of the points -> global graph (read when a bucket is made)
V2G_PIECES = 4  # pieces per scene of the views -> global graph (one-level combine)
HEADROOM = 1.04  # a new bucket's sizes over the batch's
MAX_WASTE = 1.12  # a batch reuses a bucket up to this much larger than itself (+ the fixed pads)


class BatchStats:
    """Host statistics of a batch of device-built scenes: ONE host read."""

    def __init__(self, datas):
        self.B = len(datas)
        self.ms = [int(d.x.shape[0]) for d in datas]
        self.ns = [int(d.x.shape[1]) for d in datas]
        self.Es = [int(d.x.indices.shape[1]) for d in datas]
        self.arrays = [_scene_arrays(d) for d in datas]
        rows = []
        for d, a in zip(datas, self.arrays):
            deg = (a[0][1:] - a[0][:-1]).to(torch.int64)
            cpp = d.x.cam_per_pts.view(-1).to(torch.int64)
            ppc = d.x.pts_per_cam.view(-1).to(torch.int64)
            pieces = torch.clamp((deg + PIECE - 1) // PIECE, min=1)
            rows.append(torch.stack([pieces.sum(), deg.min(), (ppc >= MIN_N_POINTS_PER_VIEW).sum(),
                                     (cpp >= MIN_N_VIEWS_PER_POINT).sum(), cpp.max()]))
        v = torch.stack(rows).tolist()
        self.pieces_s = [r[0] for r in v]
        self.pieces = sum(self.pieces_s)
        self.min_cam_deg = min(r[1] for r in v)
        self.kv = [r[2] for r in v]
        self.kp = [r[3] for r in v]
        self.max_pt_deg = max(r[4] for r in v)
        self.M, self.N, self.E = sum(self.ms), sum(self.ns), sum(self.Es)
        self.inv_v = self.M - sum(self.kv)
        self.inv_p = self.N - sum(self.kp)

    def expressible(self):
        """None, or why the static scheme cannot run this batch."""
        if self.min_cam_deg < 1:
            return "a camera without edges"
        if self.max_pt_deg > PIECE:
            return f"a point seen by {self.max_pt_deg} > {PIECE} views"
        if min(self.kv) < V2G_PIECES:
            return f"a scene with {min(self.kv)} < V2G_PIECES = {V2G_PIECES} valid views"
        if min(self.kp) < S2G_PIECES:
            return f"a scene with {min(self.kp)} < S2G_PIECES = {S2G_PIECES} valid points"
        return None


class Caps:
    """A bucket: fixed cameras / points / edges / camera pieces of the padded union of B scenes."""

    def __init__(self, B, M, N, E, inv_v, inv_p):
        self.B, self.M, self.N, self.E = B, M, N, E
        self.inv_v, self.inv_p = inv_v, inv_p
        self.S = B + 1
        self.I = -(-E // PIECE) + M  # >= sum of ceil(deg / PIECE) over any M cameras with E edges
        self.P = S2G_PIECES
        self.PV = V2G_PIECES
        self.G = math.ceil(math.sqrt(self.P))  # level-1 group size of its combine (attention._two_level)
        self.NG = -(-self.P // self.G)  # level-1 rows per scene

    def key(self):
        return (self.B, self.M, self.N, self.E, self.inv_v, self.inv_p)

    def pad(self, st):
        """(M_pad, N_pad, E_pad, pad camera pieces) for a batch, or None when the batch does not fit."""
        if (st.B, st.inv_v, st.inv_p) != (self.B, self.inv_v, self.inv_p) or min(st.kp) < self.P \
                or min(st.kv) < self.PV:
            return None
        mp, npd, ep, dI = self.M - st.M, self.N - st.N, self.E - st.E, self.I - st.pieces
        if mp < self.PV or npd < self.P or ep < 2 * npd or ep > PIECE * npd or ep < MIN_N_POINTS_PER_VIEW * mp:
            return None
        if dI < mp or ep // mp < -(-dI // mp):  # every pad camera: >= 1 piece, >= 1 edge per piece
            return None
        return mp, npd, ep, dI

    def waste_ok(self, st):
        return (self.E <= MAX_WASTE * st.E + 2 * (S2G_PIECES + 64) + 4096
                and self.N <= MAX_WASTE * st.N + S2G_PIECES + 1024)

    @classmethod
    def for_batch(cls, st):
        # >= V2G_PIECES pad cameras (the pad scene's view->global graph is split like every scene's:
        # a one-scene batch of 13 views would otherwise get 3 and no edge count could fix it)
        M = -(-max(st.M + 1 + st.M // 8, st.M + V2G_PIECES) // 8) * 8
        N = -(-(int(st.N * HEADROOM) + S2G_PIECES + 64) // 256) * 256
        E = max(int(st.E * HEADROOM), st.E + 2 * (N - st.N) + MIN_N_POINTS_PER_VIEW * (M - st.M) + 256)
        E = -(-E // 2048) * 2048
        caps = cls(st.B, M, N, E, st.inv_v, st.inv_p)
        for _ in range(1 << 16):  # grow the edges until the pads are expressible
            if caps.pad(st) is not None:
                return caps
            caps = cls(st.B, M, N, caps.E + 2048, st.inv_v, st.inv_p)
        raise RuntimeError(f"StaticBatch: no bucket found for a batch of M={st.M} N={st.N} E={st.E}")


def _inv3(Ns):
    """Closed-form inverse of [k, 3, 3] matrices (device ops, no host sync)."""
    a, b, c = Ns[:, 0, 0], Ns[:, 0, 1], Ns[:, 0, 2]
    d, e, f = Ns[:, 1, 0], Ns[:, 1, 1], Ns[:, 1, 2]
    g, h, i = Ns[:, 2, 0], Ns[:, 2, 1], Ns[:, 2, 2]
    A, B_, C = e * i - f * h, f * g - d * i, d * h - e * g
    det = a * A + b * B_ + c * C
    adj = torch.stack([A, c * h - b * i, b * f - c * e,
                       B_, a * i - c * g, c * d - a * f,
                       C, b * g - a * h, a * e - b * d], 1).view(-1, 3, 3)
    return adj / det.view(-1, 1, 1)


class StaticBatch:
    """The static input buffers of one bucket, in the shape the model reads (``.x``, ``.graph_wrappers``,
    ``.scene_of_cam``), with the plans built over them once; ``fill`` writes a batch into them."""

    def __init__(self, caps, device):
        self.caps = c = caps
        self.device = dev = device
        self.B = c.B
        S, M, N, E, I = c.S, c.M, c.N, c.E, c.I
        i32 = dict(dtype=torch.int32, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        z = lambda *shape, **kw: torch.zeros(shape, **kw)
        self.values = z(E, 2, **f32)  # the network's measurements
        self.values_loss = z(E, 2, **f32)  # the loss's (the clean scene under outlier injection)
        self.xy = z(E, 2, **f32)  # pixel measurements (compute_core_errors)
        self.indices = z(2, E, **i64)
        self.cam32, self.pt32 = z(E, **i32), z(E, **i32)
        self.cam_ptr, self.pt_ptr = z(M + 1, **i32), z(N + 1, **i32)
        self.perm, self.pos = z(E, **i32), z(E, **i32)
        self.cam_per_pts, self.pts_per_cam = z(N, 1, **i64), z(M, 1, **i64)
        self.scene_of_cam = z(M, **i64)
        self.soc32, self.sop32 = z(M, **i32), z(N, **i32)
        # one int32 buffer fed from the host per step: the global graphs' items / segments and the
        # loss's edge offsets (views below; items first, so their rows stay 16-byte aligned)
        nh = S * c.P * 4 + S * c.PV * 4 + 3 * (S + 1)
        self.hostfed = z(nh, **i32)
        o = 0
        views = {}
        for name, n, shape in (("items_s", S * c.P * 4, (S * c.P, 4)), ("items_v", S * c.PV * 4, (S * c.PV, 4)),
                               ("seg_v", S + 1, (S + 1,)), ("seg_p", S + 1, (S + 1,)), ("eoff", S + 1, (S + 1,))):
            views[name] = self.hostfed[o:o + n].view(shape)
            o += n
        self.eoff = views["eoff"]
        self.weight = torch.tensor([1.0] * c.B + [0.0], **f32)
        self.Ns_inv = torch.eye(3, **f32).repeat(M, 1, 1)
        # camera plan: I items, every camera through partial slots, one combine entry per camera
        self.items_c = z(I, 4, **i32)
        self.comb_c = z(M, 4, **i32)
        # point plan: one unsplit item per point
        self.items_p = z(N, 4, **i32)
        # global graphs: sources = valid views / points (scene-major), one segment per scene
        self.kv_cap, self.kp_cap = M - c.inv_v, N - c.inv_p
        # (all views valid / all points valid -- the usual case -- makes the sources the identity)
        self.src_v = torch.arange(M, **i32) if c.inv_v == 0 else z(self.kv_cap, **i32)
        self.src_p = torch.arange(N, **i32) if c.inv_p == 0 else z(self.kp_cap, **i32)
        self.seg_v, self.seg_p = views["seg_v"], views["seg_p"]
        self.items_v, self.items_s = views["items_v"], views["items_s"]
        self.pos_v = torch.arange(M, **i32) if self.kv_cap == M else None
        self.pos_p = torch.arange(N, **i32) if self.kp_cap == N else None
        n_slots = S * c.P
        s = torch.arange(S, **i64)
        self.comb_s = torch.stack([s, n_slots + s * c.NG, torch.full_like(s, c.NG), torch.ones_like(s)], 1).to(
            torch.int32).contiguous()
        k = torch.arange(S * c.NG, **i64)
        ks, kk = k // c.NG, k % c.NG
        self.l1_s = torch.stack([n_slots + k, ks * c.P + kk * c.G, torch.clamp(c.P - kk * c.G, max=c.G),
                                 torch.ones_like(k)], 1).to(torch.int32).contiguous()
        empty = torch.zeros((0, 4), **i32)
        pv = AttnPlan(self.cam_ptr, None, self.items_c, self.comb_c, I, M, E, E, max_piece=PIECE, combine_l1=None)
        pp = AttnPlan(self.pt_ptr, self.perm, self.items_p, empty, 0, N, E, E, max_piece=PIECE, pos=self.pos,
                      combine_l1=None)
        sv = torch.arange(S, **i64)
        self.comb_v = torch.stack([sv, sv * c.PV, torch.full_like(sv, c.PV), torch.ones_like(sv)], 1).to(
            torch.int32).contiguous()
        pg = AttnPlan(self.seg_v, self.src_v, self.items_v, self.comb_v, S * c.PV, S, self.kv_cap, M, max_piece=1 << 30,
                      pos=self.pos_v, combine_l1=None)
        ps = AttnPlan(self.seg_p, self.src_p, self.items_s, self.comb_s, n_slots, S, self.kp_cap, N,
                      max_piece=1 << 30, pos=self.pos_p, combine_l1=self.l1_s)
        self.x = SparseMat(self.values, self.indices, self.cam_per_pts, self.pts_per_cam, (M, N, 2))
        gw = {}
        for name, plan, w in (("proj2view", pv, AxialAggregationGraphWrapper(M, N, 1, self.indices, build_plan=False)),
                              ("proj2scenepoint", pp, AxialAggregationGraphWrapper(M, N, 0, self.indices,
                                                                                   build_plan=False)),
                              ("view2global", pg, None), ("scenepoint2global", ps, None)):
            plan.tag = name
            if w is None:
                w = AxialAggregationGraphWrapper.__new__(AxialAggregationGraphWrapper)
                w.device = dev
            w.plan = plan
            gw[name] = w
        self.graph_wrappers = gw
        self.scene_name = f"static{c.key()}"
        # the model's int32 edge ids and plans, cached on x under the key model.edge_index_for uses:
        # they ARE the static buffers, so a replay reads what fill() wrote
        plans = {n: w.plan for n, w in gw.items()}
        plans["_scene_of_cam"] = self.scene_of_cam
        self.x.__dict__["_gasfm_edges"] = {
            (str(dev), self.indices.data_ptr()): EdgeIndex(self.cam32, self.pt32, M, N, plans)}
        self.offsets = None
        self._out = None
        if dev.type == "cuda":
            o = _native.UnionOut()
            for k in ("indices", "cam32", "pt32", "values", "values_loss", "xy", "perm", "pos", "cam_ptr", "pt_ptr",
                      "cam_per_pts", "pts_per_cam", "soc32", "sop32", "Ns_inv", "items_c", "comb_c", "items_p"):
                setattr(o, k, getattr(self, k).data_ptr())
            o.soc = self.scene_of_cam.data_ptr()
            o.ld_indices = E
            o.piece = PIECE
            self._out = o

    @staticmethod
    def _pieces_np(seg, P):
        """P pieces per segment of seg (lengths differing by at most one, the first len % P longer),
        slot = item index: the items of an all-split plan (numpy)."""
        S = seg.shape[0] - 1
        k = np.arange(S * P)
        ks, kq = k // P, k % P
        cnt = (seg[1:] - seg[:-1])[ks]
        b2, r2 = cnt // P, cnt % P
        begin = seg[:-1][ks] + kq * b2 + np.minimum(kq, r2)
        return np.stack([ks, begin, begin + b2 + (kq < r2), k], 1)

    def _host_plans(self, st, npd):
        """The global graphs' segments / items and the edge offsets from host counts (all views and all
        points valid): int32 array laid out as self.hostfed."""
        c = self.caps
        S, P = c.S, c.P
        seg_v = np.concatenate([[0], np.cumsum(st.ms + [c.M - st.M])]).astype(np.int64)
        seg_p = np.concatenate([[0], np.cumsum(st.ns + [npd])]).astype(np.int64)
        items_s = self._pieces_np(seg_p, P)
        items_v = self._pieces_np(seg_v, c.PV)
        eo = np.concatenate([[0], np.cumsum(st.Es), [c.E]])
        return np.concatenate([items_s.ravel(), items_v.ravel(), seg_v, seg_p, eo]).astype(np.int32)

    # ------------------------------------------------------------------ per-step fill
    def fill(self, datas, st, inputs=None):
        """Write the batch (device-built scenes; ``inputs``: the network's inputs when they differ from
        the loss's scenes, e.g. outlier-injected copies with the same edges) and this bucket's pad scene
        into the static buffers: one gasfm_union_fill_scene launch per scene, one gasfm_union_fill_pad,
        one host-to-device copy of the global graphs' items.  fill_torch is the same in torch ops (the
        CPU path, and the GPU test's check of this one)."""
        c = self.caps
        if self._out is None:
            return self.fill_torch(datas, st, inputs)
        pad = c.pad(st)
        if pad is None:
            raise ValueError("StaticBatch.fill: the batch does not fit this bucket")
        mp, npd, ep, dI = pad
        inputs = datas if inputs is None else inputs
        dev = self.device
        mo = [sum(st.ms[:i]) for i in range(st.B + 1)]
        no = [sum(st.ns[:i]) for i in range(st.B + 1)]
        eo = [sum(st.Es[:i]) for i in range(st.B + 1)]
        keep = []  # operands made contiguous here stay referenced until the launches are queued
        item0 = 0
        for s, (d, din, a) in enumerate(zip(datas, inputs, st.arrays)):
            if int(din.x.indices.shape[1]) != st.Es[s]:
                raise ValueError("StaticBatch.fill: the network's input scene has other edges than the loss's")
            sc = _native.UnionScene()
            idx = d.x.indices
            if idx.dtype != torch.int64 or idx.stride(1) != 1:
                idx = idx.to(torch.int64).contiguous()
            sc.idx, sc.ld_idx = idx.data_ptr(), idx.stride(0)
            t = {"vals": din.x.values, "vals_loss": d.x.values}
            for k, v in t.items():
                t[k] = v.to(torch.float32).contiguous()
            t["cptr"], t["pptr"] = a[0].to(torch.int32).contiguous(), a[1].to(torch.int32).contiguous()
            t["perm"] = None if a[2] is None else a[2].to(torch.int32).contiguous()
            t["pos"] = None if a[3] is None else a[3].to(torch.int32).contiguous()
            t["cam_per_pts"] = d.x.cam_per_pts.to(torch.int64).contiguous()
            t["pts_per_cam"] = d.x.pts_per_cam.to(torch.int64).contiguous()
            t["Ns"] = d.Ns.to(dev, torch.float32).contiguous()
            Md = getattr(d, "_M", None)
            if Md is None:
                Md = getattr(d, "M", None)
            if Md is not None:
                Md = Md.to(dev, torch.float32)
                if Md.stride(1) != 1:
                    Md = Md.contiguous()
                sc.ldM = Md.stride(0)
            t["M"] = Md
            for k, v in t.items():
                setattr(sc, k, None if v is None else v.data_ptr())
            keep.append((idx, t))
            sc.E, sc.m, sc.n = st.Es[s], st.ms[s], st.ns[s]
            sc.e0, sc.c0, sc.p0, sc.item0, sc.scene = eo[s], mo[s], no[s], item0, s
            item0 += st.pieces_s[s]
            _native.union_fill_scene(sc, self._out, self.values)
        pd = _native.UnionPad()
        pd.M, pd.N, pd.E, pd.mp, pd.npd, pd.ep, pd.dI, pd.item0, pd.scene = st.M, st.N, st.E, mp, npd, ep, dI, item0, st.B
        _native.union_fill_pad(pd, self._out, self.values)
        self.offsets = (mo, no, eo)
        if c.inv_v == 0 and c.inv_p == 0:
            # a fresh pinned block per step: the caching host allocator keeps it until the copy ran
            self.hostfed.copy_(torch.from_numpy(self._host_plans(st, npd)).pin_memory(), non_blocking=True)
        else:
            self.eoff.copy_(torch.tensor(eo + [c.E], dtype=torch.int32).to(dev))
            self._global_plans_torch()

    def fill_torch(self, datas, st, inputs=None):
        """``fill`` in torch ops."""
        c = self.caps
        pad = c.pad(st)
        if pad is None:
            raise ValueError("StaticBatch.fill: the batch does not fit this bucket")
        mp, npd, ep, dI = pad
        inputs = datas if inputs is None else inputs
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        mo = [sum(st.ms[:i]) for i in range(st.B + 1)]
        no = [sum(st.ns[:i]) for i in range(st.B + 1)]
        eo = [sum(st.Es[:i]) for i in range(st.B + 1)]
        M, N, E = st.M, st.N, st.E
        for s, (d, din, a) in enumerate(zip(datas, inputs, st.arrays)):
            if int(din.x.indices.shape[1]) != st.Es[s]:
                raise ValueError("StaticBatch.fill: the network's input scene has other edges than the loss's")
            e0, e1, c0, c1, p0, p1 = eo[s], eo[s + 1], mo[s], mo[s + 1], no[s], no[s + 1]
            idx = d.x.indices
            self.indices[0, e0:e1].copy_(idx[0])
            self.indices[0, e0:e1] += c0
            self.indices[1, e0:e1].copy_(idx[1])
            self.indices[1, e0:e1] += p0
            self.values[e0:e1].copy_(din.x.values)
            self.values_loss[e0:e1].copy_(d.x.values)
            self.cam_ptr[c0:c1].copy_(a[0][:-1])
            self.cam_ptr[c0:c1] += e0
            self.pt_ptr[p0:p1].copy_(a[1][:-1])
            self.pt_ptr[p0:p1] += e0
            perm, pos = a[2], a[3]
            if perm is None:
                self.perm[e0:e1].copy_(torch.arange(e0, e1, **i32))
                self.pos[e0:e1].copy_(self.perm[e0:e1])
            else:
                self.perm[e0:e1].copy_(perm)
                self.perm[e0:e1] += e0
                self.pos[e0:e1].copy_(pos)
                self.pos[e0:e1] += e0
            self.cam_per_pts[p0:p1].copy_(d.x.cam_per_pts)
            self.pts_per_cam[c0:c1].copy_(d.x.pts_per_cam)
            Md = getattr(d, "_M", None)
            if Md is None:
                Md = getattr(d, "M", None)
            if Md is not None:
                Md = Md.to(dev)
                self.xy[e0:e1, 0].copy_(Md[2 * idx[0], idx[1]])
                self.xy[e0:e1, 1].copy_(Md[2 * idx[0] + 1, idx[1]])
        self.Ns_inv[:M].copy_(_inv3(torch.cat([d.Ns.to(dev, torch.float32) for d in datas])))
        # the pad scene: mp cameras, npd points, ep edges, cam-major and point-sorted
        ar = lambda n: torch.arange(n, **i64)
        degc = ep // mp + (ar(mp) < ep % mp).to(torch.int64)
        degp = ep // npd + (ar(npd) < ep % npd).to(torch.int64)
        pc = M + torch.repeat_interleave(ar(mp), degc, output_size=ep)
        pp = N + torch.repeat_interleave(ar(npd), degp, output_size=ep)
        self.indices[0, E:].copy_(pc)
        self.indices[1, E:].copy_(pp)
        self.values[E:].zero_()
        self.values_loss[E:].zero_()
        self.xy[E:].zero_()
        self.cam_ptr[M:c.M].copy_(E + torch.cumsum(degc, 0) - degc)
        self.cam_ptr[c.M] = c.E
        self.pt_ptr[N:c.N].copy_(E + torch.cumsum(degp, 0) - degp)
        self.pt_ptr[c.N] = c.E
        self.perm[E:].copy_(torch.arange(E, c.E, **i32))
        self.pos[E:].copy_(self.perm[E:])
        self.cam_per_pts[N:, 0].copy_(degp)
        self.pts_per_cam[M:, 0].copy_(degc)
        self.Ns_inv[M:].copy_(torch.eye(3, dtype=torch.float32, device=dev))
        self.cam32.copy_(self.indices[0])
        self.pt32.copy_(self.indices[1])
        # scene maps and edge offsets: one host-to-device copy of the small host lists
        h = torch.tensor(sum(([s] * m for s, m in enumerate(st.ms)), []) + [st.B] * mp + st.ns + [npd] + eo + [c.E],
                         dtype=torch.int64)
        h = h.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else h.to(dev)
        soc = h[:c.M]
        self.scene_of_cam.copy_(soc)
        self.soc32.copy_(soc)
        sop = torch.repeat_interleave(torch.arange(c.S, **i64), h[c.M:c.M + c.S], output_size=c.N)
        self.sop32.copy_(sop)
        self.eoff.copy_(h[c.M + c.S:])
        self.offsets = (mo, no, eo)
        # camera plan: real cameras ceil(deg / PIECE) pieces, pad cameras the remaining dI
        cptr = self.cam_ptr.to(torch.int64)
        ln = cptr[1:] - cptr[:-1]
        pieces = torch.clamp((ln + PIECE - 1) // PIECE, min=1)
        pieces[M:] = dI // mp + (ar(mp) < dI % mp).to(torch.int64)
        seg = torch.repeat_interleave(ar(c.M), pieces, output_size=c.I)
        first = torch.cumsum(pieces, 0) - pieces
        q = ar(c.I) - first[seg]
        base, rem = ln // pieces, ln % pieces
        begin = cptr[:-1][seg] + q * base[seg] + torch.minimum(q, rem[seg])
        end = begin + base[seg] + (q < rem[seg]).to(torch.int64)
        self.items_c.copy_(torch.stack([seg, begin, end, ar(c.I)], 1))
        self.comb_c.copy_(torch.stack([ar(c.M), first, pieces, torch.ones_like(pieces)], 1))
        # point plan
        pptr = self.pt_ptr.to(torch.int64)
        self.items_p.copy_(torch.stack([ar(c.N), pptr[:-1], pptr[1:], torch.full((c.N,), -1, **i64)], 1))
        self._global_plans_torch()

    def _global_plans_torch(self):
        """view2global / scenepoint2global segments and items from the filled counts (torch ops)."""
        c = self.caps
        i64 = dict(dtype=torch.int64, device=self.device)
        sop = self.sop32.to(torch.int64)
        # view2global: V2G_PIECES pieces per scene over its valid views, every scene split
        valid_v = self.pts_per_cam.view(-1) >= MIN_N_POINTS_PER_VIEW
        self.src_v.copy_(torch.nonzero_static(valid_v, size=self.kv_cap).view(-1))
        cv = torch.zeros(c.S, **i64).index_add_(0, self.scene_of_cam, valid_v.to(torch.int64))
        self.seg_v[1:].copy_(torch.cumsum(cv, 0))
        self.items_v.copy_(self._pieces_torch(self.seg_v.to(torch.int64), c.PV))
        # scenepoint2global: S2G_PIECES pieces per scene, every scene split
        valid_p = self.cam_per_pts.view(-1) >= MIN_N_VIEWS_PER_POINT
        self.src_p.copy_(torch.nonzero_static(valid_p, size=self.kp_cap).view(-1))
        cp = torch.zeros(c.S, **i64).index_add_(0, sop, valid_p.to(torch.int64))
        self.seg_p[1:].copy_(torch.cumsum(cp, 0))
        self.items_s.copy_(self._pieces_torch(self.seg_p.to(torch.int64), c.P))

    @staticmethod
    def _pieces_torch(seg, P):
        """_pieces_np in torch ops on seg's device."""
        S = seg.shape[0] - 1
        k = torch.arange(S * P, dtype=torch.int64, device=seg.device)
        ks, kq = k // P, k % P
        cnt = (seg[1:] - seg[:-1])[ks]
        b2, r2 = cnt // P, cnt % P
        begin = seg[:-1][ks] + kq * b2 + torch.minimum(kq, r2)
        return torch.stack([ks, begin, begin + b2 + (kq < r2).to(torch.int64), k], 1)

    def split(self, pred):
        """Per-scene prediction dicts (views into the union outputs) of the last fill."""
        mo, no, _ = self.offsets
        return [{"Ps_norm": pred["Ps_norm"][mo[i]:mo[i + 1]], "pts3D": pred["pts3D"][:, no[i]:no[i + 1]]}
                for i in range(self.B)]


class BatchLossFn(torch.autograd.Function):
    """sum over the real scenes of ESFMLoss(pred, scene) on a StaticBatch (gasfm_esfm_seg_fwd / _bwd):
    the eager step's ``sum(lossf(p, d) for ...)`` with fixed launch geometry."""

    @staticmethod
    def forward(ctx, Ps, pts3D, sb, conf):
        margin, hinge_w, hinge, equalize, valid_only = conf
        P = Ps.reshape(Ps.shape[0], 12).contiguous()
        X = pts3D.contiguous()
        loss, tot = _native.esfm_seg_fwd(sb.cam32, sb.pt32, sb.values_loss, sb.eoff, sb.weight, P, X, margin,
                                         hinge_w, hinge)
        ctx.save_for_backward(P, X, tot)
        ctx.sb, ctx.conf = sb, conf
        return loss.view(())

    @staticmethod
    def backward(ctx, dloss):
        P, X, tot = ctx.saved_tensors
        sb = ctx.sb
        margin, hinge_w, hinge, equalize, valid_only = ctx.conf
        dP, dX = torch.empty_like(P), torch.empty_like(X)
        dloss = dloss.reshape(1).to(torch.float32).contiguous()
        _native.esfm_seg_bwd(sb.cam_ptr, sb.pt_ptr, sb.perm, sb.cam32, sb.pt32, sb.values_loss, sb.eoff, sb.soc32,
                             sb.sop32, sb.weight, P, X, margin, hinge_w, hinge, equalize, valid_only, dloss, tot, dP,
                             dX)
        return dP.view(-1, 3, 4), dX, None, None


def batch_loss(pred, sb, lossf):
    return BatchLossFn.apply(pred["Ps_norm"], pred["pts3D"], sb, lossf.kernel_conf())


def batch_repro_errors(pred, sb):
    """[S, 2] per-scene (sum, count) of the non-NaN reprojection errors (compute_core_errors' our_repro
    = sum / count) of a StaticBatch, on the device."""
    Ps = pred["Ps_norm"].detach()
    P = torch.bmm(sb.Ns_inv, Ps).reshape(-1, 12).contiguous()
    return _native.reproj_error_seg(sb.cam32, sb.pt32, sb.xy, sb.eoff, sb.caps.S, P,
                                    pred["pts3D"].detach().float().contiguous())


class StaticTrainer:
    """Forward + ESFMLoss + backward of a batch of scenes as a replayed hipGraph per bucket.

    ``step(datas, inputs=None)`` leaves this batch's gradients in ``p.grad`` (as zero_grad + the eager
    union's loss.backward()) and returns (loss 0-d tensor, per-scene our_repro errors list).
    Config 5: ``inputs`` = the outlier-injected scenes the network sees, ``datas`` the clean ones the
    loss and the errors use (train.py:73-90).

    optimizer: stepped after the gradients (train.py:97-100).  With ``capturable=True`` (torch's
    Adam / AdamW) its step is captured too, one graph per bucket over that bucket's gradient
    tensors, once its state exists (the first step of a run is eager); a Python-float learning rate
    is then fixed at capture (pass a tensor lr to schedule it)."""

    def __init__(self, net, lossf, warmup=2, optimizer=None, max_buckets=32):
        """max_buckets: the least recently used bucket (its graphs and buffers) is dropped beyond it."""
        self.net, self.lossf = net, lossf
        self.max_buckets = max_buckets
        self.optimizer = optimizer
        self.opt_graphs = 0
        self.params = [p for p in net.parameters() if p.requires_grad]
        self.buckets = {}
        self.pool = torch.cuda.graph_pool_handle()
        self.warmup = warmup
        self.captures = 0
        self.eager_steps = 0
        self.fallbacks = []
        self.profile = None  # a dict: per-phase host seconds (stats, fill, replay, optimizer), synchronised

    def _bucket(self, st, dev):
        best = None
        for b in self.buckets.values():
            c = b[0].caps
            if c.pad(st) is not None and c.waste_ok(st) and (best is None or c.E < best[0].caps.E):
                best = b
        if best is not None:
            key = best[0].caps.key()
            self.buckets[key] = self.buckets.pop(key)  # most recently used last
            return best, False
        caps = Caps.for_batch(st)
        best = self.buckets.pop(caps.key(), None)
        if best is None:
            best = [StaticBatch(caps, dev), None]
            while len(self.buckets) >= self.max_buckets:  # drop the least recently used
                self.buckets.pop(next(iter(self.buckets)))
        self.buckets[caps.key()] = best
        return best, True

    def _eager(self, datas, inputs):
        from .batch import SceneBatch
        from . import evaluation
        self.eager_steps += 1
        for p in self.params:
            p.grad = None
        union = SceneBatch(inputs)
        preds = union.split(self.net(union))
        loss = sum(self.lossf(p, d) for p, d in zip(preds, datas))
        loss.backward()
        errs = [float(evaluation.reprojection_error_mean(d, p)) for p, d in zip(preds, datas)]
        return loss.detach(), errs

    def _optimizer_step(self, b):
        opt = self.optimizer
        if len(b) > 3:
            b[3].replay()
        elif b[1].captured and opt.defaults.get("capturable") and all(p in opt.state for p in self.params):
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with gc_paused(), torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local"):
                opt.step()
            g.replay()
            b.append(g)
            self.opt_graphs += 1
        else:
            opt.step()
        self._refresh_if_bf16()

    def _refresh_if_bf16(self):
        """Re-round the bf16 weight shadows after every optimizer step, captured or eager: a replayed
        graph reads dense._SHADOWS without a version check."""
        if getattr(self.net, "_projection_precision", "fp32") == "bf16":
            self.net.refresh_weight_shadows()

    def _tick(self, phase):
        if self.profile is not None:
            torch.cuda.synchronize()
            t = time.perf_counter()
            if phase is not None:
                self.profile[phase] = self.profile.get(phase, 0.0) + t - self._t
            self._t = t

    @staticmethod
    def errors(tot):
        """Per-scene our_repro from the [B, 2] (sum, count) device tensor step(read_errors=False) returns."""
        return [a / b if b else float("nan") for a, b in tot.tolist()]

    def step(self, datas, inputs=None, stats=None, read_errors=True):
        """stats: the inputs' BatchStats when already taken (e.g. on the stream that prepared the batch);
        read_errors=False: return the per-scene (sum, count) error tensor instead of reading it (no host
        synchronisation: the caller can prepare the next batch while this one replays; ``errors``
        converts it)."""
        from .graph_step import CapturedStep
        inputs = datas if inputs is None else inputs
        self._tick(None)
        st = BatchStats(inputs) if stats is None else stats
        why = st.expressible()
        if why is not None:
            self.fallbacks.append(why)
            loss, errs = self._eager(datas, inputs)
            if self.optimizer is not None:
                self.optimizer.step()
                self._refresh_if_bf16()
            if not read_errors:
                errs = torch.tensor([[e, 1.0] for e in errs], dtype=torch.float32)
            return loss, errs
        dev = inputs[0].x.values.device
        b, _ = self._bucket(st, dev)
        sb = b[0]
        self._tick("stats")
        sb.fill(datas, st, inputs)
        self._tick("fill")
        out = {}

        def fwd_bwd():
            pred = self.net(sb)
            loss = batch_loss(pred, sb, self.lossf)
            out["err"] = batch_repro_errors(pred, sb)
            loss.backward()
            return loss

        if b[1] is None:
            b[1] = CapturedStep(fwd_bwd, self.params, warmup=self.warmup if not self.captures else 1,
                                pool=self.pool)
            b.append(out)
            self.captures += 1
            if not b[1].captured:
                self.fallbacks.append(b[1].fallback_reason)
        loss = b[1]()
        self._tick("replay" if b[1].captured else "eager")
        if self.optimizer is not None:
            self._optimizer_step(b)
            self._tick("optimizer")
        err = b[2]["err"][:st.B]
        if not read_errors:
            return loss, err.clone()  # the static buffer is overwritten by the next replay
        return loss, self.errors(err)
