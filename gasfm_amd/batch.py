"""Several scenes in one forward: the disjoint union of their graphs (BASELINE config 3's batch).

train.py (:60-96) runs the model once per scene of a batch and sums the losses before one
backward.  Every scene's graph is small (10-20 sampled views), so each forward + backward is
~2,000 short kernels whose cost is the host's (Python / autograd / launch), not the GPU's:
``profiles/r1_train_step_bench.txt`` measured 158 ms for 4 scenes.  The scenes do not interact,
so running them as ONE graph -- cameras, points and edges concatenated with offsets, one global
node per scene -- computes exactly the per-scene forwards (every attention is per destination;
every LayerNorm / MLP is per row) in one pass of launches:

  proj2view / proj2scenepoint   the union's camera / point segments (edge ranges offset)
  view2global / scenepoint2global   B destination segments (scene s's valid views / points)
  global rows                   [B, G] through the multi-row paths (dense.py falls back from the
                                single-row gvec kernels to row-batched GEMMs)
  projection update             the per-edge global term lin_global(g_s) is folded into the
                                per-camera term (each camera belongs to one scene):
                                Sv'[c] = Sv[c] + Sg[scene(c)], then the edge kernels run as for
                                one scene (model.GraphAttnSfMLayer, ``_scene_of_cam``)

``forward_batch(net, datas)`` returns the per-scene prediction dicts (views of the union
outputs), so the loss is the reference's per scene; their sum back-propagates once.  Results
equal the per-scene forwards up to fp32 summation order (tests/test_gpu_batch.py).
"""
import torch

from .attention import DEFAULT_MAX_PIECE
from .scene import MIN_N_POINTS_PER_VIEW, MIN_N_VIEWS_PER_POINT, AxialAggregationGraphWrapper, SparseMat
from .scene_device import _piece_counts_host, _piece_stats, _plan


def _scene_arrays(d):
    """(cam_ptr, pt_ptr, perm, pos, point-sorted flag) of one scene: from the device scene build when
    the scene's graph wrappers were never built (scene_device: they are built on first use), else
    from its plans.  The flag is a device bool or a Python bool."""
    b = d.__dict__.get("_scene_build")
    if b is not None and "graph_wrappers" not in d.__dict__:
        pt = b["pt"]
        srt = (pt[1:] >= pt[:-1]).all() if pt.shape[0] > 1 else True
        return b["cam_ptr"], b["pt_ptr"], b["perm"], b["pos"], srt
    gw = d.graph_wrappers
    p = gw["proj2scenepoint"].plan
    return gw["proj2view"].plan.seg_ptr, p.seg_ptr, p.perm, p.pos, p.perm is None


class SceneBatch:
    """The union graph of several device-built scenes (each with .x and plan-carrying wrappers)."""

    def __init__(self, datas, max_piece=None):
        if not datas:
            raise ValueError("SceneBatch: no scenes")
        dev = datas[0].x.values.device
        self.datas = list(datas)
        self.B = len(datas)
        ms = [d.x.shape[0] for d in datas]
        ns = [d.x.shape[1] for d in datas]
        Es = [int(d.x.indices.shape[1]) for d in datas]
        self.cam_off = [sum(ms[:i]) for i in range(self.B + 1)]
        self.pt_off = [sum(ns[:i]) for i in range(self.B + 1)]
        self.edge_off = [sum(Es[:i]) for i in range(self.B + 1)]
        M, N, E = self.cam_off[-1], self.pt_off[-1], self.edge_off[-1]
        i64 = dict(dtype=torch.int64, device=dev)
        cam = torch.cat([d.x.indices[0].to(dev) + self.cam_off[i] for i, d in enumerate(datas)])
        pt = torch.cat([d.x.indices[1].to(dev) + self.pt_off[i] for i, d in enumerate(datas)])
        vals = torch.cat([d.x.values for d in datas])
        cpp = torch.cat([d.x.cam_per_pts.to(dev) for d in datas])
        ppc = torch.cat([d.x.pts_per_cam.to(dev) for d in datas])
        self.x = SparseMat(vals, torch.stack([cam, pt]), cpp, ppc, (M, N, vals.shape[1]))
        self.device = dev
        self.scene_name = "batch(" + ",".join(getattr(d, "scene_name", "?") for d in datas) + ")"
        self.scene_of_cam = torch.repeat_interleave(torch.arange(self.B, **i64),
                                                    torch.tensor(ms, **i64)).contiguous()
        arrs = [_scene_arrays(d) for d in datas]
        mp = DEFAULT_MAX_PIECE if max_piece is None else max_piece

        def cat_ptr(parts):
            parts = [q.to(dev, torch.int64) for q in parts]
            return torch.cat([parts[0]] + [q[1:] + self.edge_off[i] for i, q in enumerate(parts) if i > 0]
                             ).to(torch.int32).contiguous()

        cam_ptr, pt_ptr = cat_ptr([a[0] for a in arrs]), cat_ptr([a[1] for a in arrs])
        # every host scalar of the union's plans in ONE read: per-scene point-sortedness, valid view /
        # point counts per scene, the piece statistics of the two edge plans
        valid_v = ppc.view(-1) >= MIN_N_POINTS_PER_VIEW
        valid_p = cpp.view(-1) >= MIN_N_VIEWS_PER_POINT
        scene_of_pt = torch.repeat_interleave(torch.arange(self.B, **i64), torch.tensor(ns, **i64))
        cnt_v = torch.zeros(self.B, **i64).index_add_(0, self.scene_of_cam, valid_v.to(torch.int64))
        cnt_p = torch.zeros(self.B, **i64).index_add_(0, scene_of_pt, valid_p.to(torch.int64))
        srt = torch.stack([torch.as_tensor(a[4], device=dev).to(torch.int64) for a in arrs])
        st_c = _piece_stats((cam_ptr[1:] - cam_ptr[:-1]).to(torch.int64), mp)[3]
        st_p = _piece_stats((pt_ptr[1:] - pt_ptr[:-1]).to(torch.int64), mp)[3]
        vals_h = torch.cat([srt, cnt_v, cnt_p, st_c, st_p]).tolist()
        B = self.B
        sorted_h, cv, cp = vals_h[:B], vals_h[B:2 * B], vals_h[2 * B:3 * B]
        indices = torch.stack([cam, pt])
        p2v = AxialAggregationGraphWrapper(M, N, 1, indices, build_plan=False)
        p2s = AxialAggregationGraphWrapper(M, N, 0, indices, build_plan=False)
        p2v.plan = _plan(cam_ptr, None, None, M, E, E, mp, "proj2view", counts=vals_h[3 * B:3 * B + 4])

        def cat_perm(k):
            out = []
            for i, a in enumerate(arrs):
                q = a[k] if not sorted_h[i] and a[k] is not None else torch.arange(Es[i], dtype=torch.int32,
                                                                                     device=dev)
                out.append(q.to(dev, torch.int32) + self.edge_off[i])
            return torch.cat(out).contiguous()

        perm, pos = (None, None) if all(sorted_h) else (cat_perm(2), cat_perm(3))
        p2s.plan = _plan(pt_ptr, perm, pos, N, E, E, mp, "proj2scenepoint", counts=vals_h[3 * B + 4:3 * B + 8])
        # global graphs: B targets, scene s's sources (valid views / points, union indices) in segment s
        gw = {}
        for name, valid, counts, rows, tgt_dim in (("view2global", valid_v, cv, M, 0),
                                                  ("scenepoint2global", valid_p, cp, N, 1)):
            k = int(sum(counts))
            s_all = torch.nonzero_static(valid, size=k).view(-1)
            ct = torch.tensor(counts, **i64)
            seg_ptr = torch.zeros(B + 1, **i64)
            seg_ptr[1:] = torch.cumsum(ct, 0)
            tgt = torch.repeat_interleave(torch.arange(B, **i64), ct, output_size=k)
            vi = torch.stack([s_all, tgt]) if tgt_dim == 0 else torch.stack([tgt, s_all])
            w = AxialAggregationGraphWrapper(M if tgt_dim == 0 else B, B if tgt_dim == 0 else N,
                                             tgt_dim, vi, build_plan=False)
            piece = 8 if name == "view2global" else min(256, max(16, -(-max(counts) // 4096)))
            w.plan = _plan(seg_ptr.to(torch.int32).contiguous(), s_all.to(torch.int32).contiguous(), None, B, k,
                           rows, piece, name, counts=_piece_counts_host(counts, piece))
            gw[name] = w
        self.graph_wrappers = {"proj2view": p2v, "proj2scenepoint": p2s, **gw}

    def split(self, pred):
        """Per-scene prediction dicts (views into the union outputs)."""
        out = []
        for i in range(self.B):
            d = {}
            if "Ps_norm" in pred:
                d["Ps_norm"] = pred["Ps_norm"][self.cam_off[i]:self.cam_off[i + 1]]
            if "pts3D" in pred:
                d["pts3D"] = pred["pts3D"][:, self.pt_off[i]:self.pt_off[i + 1]]
            if "depths" in pred:
                dep = pred["depths"]
                x = self.datas[i].x
                d["depths"] = SparseMat(dep.values[self.edge_off[i]:self.edge_off[i + 1]], x.indices, x.cam_per_pts,
                                        x.pts_per_cam, [x.shape[0], x.shape[1], 1])
            out.append(d)
        return out


def forward_batch(net, datas, max_piece=None):
    """net(d) for every d in datas, as one forward over the union graph: list of prediction dicts."""
    batch = SceneBatch(datas, max_piece=max_piece)
    return batch.split(net(batch))
