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

from .scene import AxialAggregationGraphWrapper, SparseMat
from .scene_device import _plan


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
        pw = [d.graph_wrappers for d in datas]
        mp = max(w["proj2view"].plan.max_piece for w in pw)

        def cat_ptr(name):
            parts = [w[name].plan.seg_ptr.to(torch.int64) for w in pw]
            return torch.cat([parts[0]] + [p[1:] + self.edge_off[i] for i, p in enumerate(parts) if i > 0]
                             ).to(torch.int32).contiguous()

        def cat_perm(attr):
            out = []
            for i, w in enumerate(pw):
                p = getattr(w["proj2scenepoint"].plan, attr)
                if p is None:
                    p = torch.arange(Es[i], dtype=torch.int32, device=dev)
                out.append(p.to(torch.int32) + self.edge_off[i])
            return torch.cat(out).contiguous()

        indices = torch.stack([cam, pt])
        p2v = AxialAggregationGraphWrapper(M, N, 1, indices, build_plan=False)
        p2s = AxialAggregationGraphWrapper(M, N, 0, indices, build_plan=False)
        p2v.plan = _plan(cat_ptr("proj2view"), None, None, M, E, E, mp, "proj2view")
        sorted_pt = all(w["proj2scenepoint"].plan.perm is None for w in pw)
        perm, pos = (None, None) if sorted_pt else (cat_perm("perm"), cat_perm("pos"))
        p2s.plan = _plan(cat_ptr("proj2scenepoint"), perm, pos, N, E, E, mp, "proj2scenepoint")
        # global graphs: B targets, scene s's sources (valid views / points) in segment s
        vv = [w["view2global"].valid_indices[0].to(dev) + self.cam_off[i] for i, w in enumerate(pw)]
        vp = [w["scenepoint2global"].valid_indices[1].to(dev) + self.pt_off[i] for i, w in enumerate(pw)]
        gw = {}
        for name, src, rows, tgt_dim in (("view2global", vv, M, 0), ("scenepoint2global", vp, N, 1)):
            counts = torch.tensor([int(s.shape[0]) for s in src], **i64)
            seg_ptr = torch.zeros(self.B + 1, **i64)
            seg_ptr[1:] = torch.cumsum(counts, 0)
            s_all = torch.cat(src).contiguous()
            tgt = torch.repeat_interleave(torch.arange(self.B, **i64), counts)
            vi = torch.stack([s_all, tgt]) if tgt_dim == 0 else torch.stack([tgt, s_all])
            w = AxialAggregationGraphWrapper(M if tgt_dim == 0 else self.B, self.B if tgt_dim == 0 else N,
                                             tgt_dim, vi, build_plan=False)
            k = int(s_all.shape[0])
            piece = 8 if name == "view2global" else min(256, max(16, -(-max(int(c) for c in counts) // 4096)))
            w.plan = _plan(seg_ptr.to(torch.int32).contiguous(), s_all.to(torch.int32).contiguous(), None, self.B, k,
                           rows, piece, name)
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
