"""ESFMLoss over the visibility edges (csrc/esfm_loss.hip).

Drop-in for the reference's ``loss_functions.ESFMLoss`` (code/loss_functions.py:69-123): same
constructor (reads ``loss.infinity_pts_margin``, ``loss.pts_grad_equalization_pre_perspective_divide``,
``loss.normalize_grad_wrt_valid_projections_only``, ``loss.hinge_loss``, ``loss.hinge_loss_weight``
and asserts both heads are enabled), same ``forward(pred_dict, data, epoch=None)`` returning the
scalar loss, and the same gradients, including the ones the reference's gradient hook on the
projections imposes (loss_functions.py:104-113).

The reference projects every point into every camera (``Ps @ pts3D``: [m, 3, n], 2.4 GB at
m = 1000, n = 200k) and masks with the dense valid-observation matrix; here only the E observed
(camera, point) pairs -- the same edges the network runs on -- are projected:
  forward   one kernel -> per-workgroup (sum of loss terms, #valid-depth) -> colsum
  backward  one workgroup per camera (dPs) + one thread per point (dpts3D), no atomics
``#valid-depth`` stays on the device: the reference's ``.item()`` host sync (loss_functions.py:107)
is gone, so the loss can sit inside a captured step.

The measurement of edge e is ``data.x.values[e]``: M2sparse(normalize=True) (dataset_utils.py:116)
stores exactly the entries of ``data.norm_M`` (geo_utils.normalize_M, geo_utils.py:689) at the
valid positions, in the same cam-major order as ``data.x.indices``.
"""
import torch

from . import _native


class ESFMLossFn(torch.autograd.Function):
    """(Ps [m, 3, 4], pts3D [4, n]) -> mean over the edges of the per-edge loss term."""

    @staticmethod
    def forward(ctx, Ps, pts3D, edges, vals, cam_ptr, pt_ptr, pt_perm, conf, shard=None, E_global=None):
        """shard (gasfm_amd.distributed.ShardContext) / E_global: point-sharded scene.  Every rank
        holds all cameras and its own points with ALL their edges, so the loss is the global one
        from (sum of terms, #valid-depth) all-reduced over the ranks and divided by the global
        edge count; backward: dpts3D is rank-local and complete, dPs is summed over the ranks."""
        margin, hinge_w, hinge, equalize, valid_only = conf
        cam, pt = edges
        m = Ps.shape[0]
        P = Ps.reshape(m, 12).contiguous()
        X = pts3D.contiguous()
        part = torch.empty((_native.esfm_part_rows(cam.shape[0]), 2), dtype=torch.float32, device=X.device)
        _native.esfm_fwd(cam, pt, vals, P, X, margin, hinge_w, hinge, part)
        tot = _native.colsum(part)  # (sum of terms, #valid-depth)
        E = cam.shape[0]
        if shard is not None:
            tot = shard.all_reduce_(tot)
            E = int(E_global)
        ctx.save_for_backward(P, X, cam, pt, vals, cam_ptr, pt_ptr, pt_perm, tot)
        ctx.conf, ctx.shard, ctx.E = conf, shard, E
        return tot[0] / E

    @staticmethod
    def backward(ctx, dloss):
        P, X, cam, pt, vals, cam_ptr, pt_ptr, pt_perm, tot = ctx.saved_tensors
        margin, hinge_w, hinge, equalize, valid_only = ctx.conf
        dP, dX = torch.empty_like(P), torch.empty_like(X)
        dloss = dloss.reshape(1).to(torch.float32).contiguous()
        # E_norm = the global edge count on a sharded scene: the un-equalized terms and the equalized
        # (normalize(G) / E) branch both divide by it, as loss_functions.py:110 divides by sum(valid_pts)
        _native.esfm_bwd(cam_ptr, pt_ptr, pt_perm, cam, pt, vals, P, X, margin, hinge_w, hinge, equalize, valid_only,
                         dloss, tot, dP, dX, E_norm=ctx.E)
        if ctx.shard is not None:
            ctx.shard.all_reduce_(dP)
        return dP.view(-1, 3, 4), dX, None, None, None, None, None, None, None, None


def scene_csr(data):
    """(cache dict, camera CSR, point CSR, point-order edge ids or None) of a scene: from the device
    scene build while its graph wrappers are not built (scene_device builds them on first use), else
    from the network's own plans (proj2view: camera segments over the cam-major edges;
    proj2scenepoint: point segments with perm = edge ids in point order).  The cache dict lives as
    long as that source (per device)."""
    b = data.__dict__.get("_scene_build")
    if b is not None and "graph_wrappers" not in data.__dict__:
        return b.setdefault("caches", {}), b["cam_ptr"], b["pt_ptr"], b["perm"]
    gw = data.graph_wrappers
    pv, ps = gw["proj2view"].plan, gw["proj2scenepoint"].plan
    if pv.perm is not None:
        raise ValueError("ESFMLoss: proj2view plan must cover cam-major sorted edges")
    if "_caches" not in pv.__dict__:
        pv._caches = {}
    return pv._caches, pv.seg_ptr, ps.seg_ptr, ps.perm


def _edge_tensors(data):
    """int32 (cam, pt), contiguous float32 values and the camera / point CSRs (scene_csr).  The int32
    indices are cached, keyed on the index tensor's storage and version."""
    caches, cam_ptr, pt_ptr, pt_perm = scene_csr(data)
    idx = data.x.indices
    key = (idx.data_ptr(), idx._version, tuple(idx.shape))  # an in-place edit of the indices invalidates it
    cache = caches.get("esfm_edges")
    if cache is None or cache[0] != key:
        cache = (key, (idx[0].to(torch.int32).contiguous(), idx[1].to(torch.int32).contiguous()))
        caches["esfm_edges"] = cache
    vals = data.x.values
    if vals.dtype != torch.float32 or not vals.is_contiguous():
        vals = vals.float().contiguous()
    return cache[1], vals, cam_ptr, pt_ptr, pt_perm


class ESFMLoss(torch.nn.Module):
    def __init__(self, conf):
        super().__init__()
        assert conf.get_bool("model.view_head.enabled", default=False)
        assert conf.get_bool("model.scenepoint_head.enabled", default=False)
        self.infinity_pts_margin = conf.get_float("loss.infinity_pts_margin")
        self.pts_grad_equalization_pre_perspective_divide = conf.get_bool(
            "loss.pts_grad_equalization_pre_perspective_divide")
        self.normalize_grad_wrt_valid_projections_only = False
        if self.pts_grad_equalization_pre_perspective_divide:
            self.normalize_grad_wrt_valid_projections_only = conf.get_bool(
                "loss.normalize_grad_wrt_valid_projections_only")
        self.hinge_loss = conf.get_bool("loss.hinge_loss")
        self.hinge_loss_weight = conf.get_float("loss.hinge_loss_weight") if self.hinge_loss else 0

    def kernel_conf(self):
        return (float(self.infinity_pts_margin), float(self.hinge_loss_weight), bool(self.hinge_loss),
                bool(self.pts_grad_equalization_pre_perspective_divide),
                bool(self.normalize_grad_wrt_valid_projections_only))

    def forward(self, pred_dict, data, epoch=None):
        Ps, pts3D = pred_dict["Ps_norm"], pred_dict["pts3D"]
        for t, name, shape in ((Ps, "Ps_norm", (3, 4)), (pts3D, "pts3D", None)):
            if not t.is_cuda or t.dtype != torch.float32:
                raise TypeError(f"ESFMLoss: {name} must be a float32 CUDA tensor (no CPU fallback)")
        if Ps.dim() != 3 or tuple(Ps.shape[1:]) != (3, 4) or pts3D.dim() != 2 or pts3D.shape[0] != 4:
            raise ValueError(f"ESFMLoss: expected Ps_norm [m, 3, 4] and pts3D [4, n], got {tuple(Ps.shape)}, "
                             f"{tuple(pts3D.shape)}")
        edges, vals, cam_ptr, pt_ptr, pt_perm = _edge_tensors(data)
        if edges[0].shape[0] == 0:
            raise ValueError("ESFMLoss: no valid observations (the reference's mean would be NaN)")
        shard = getattr(data, "shard", None)
        E_global = getattr(data, "n_edges_global", None)
        if shard is not None and E_global is None:
            raise ValueError("ESFMLoss: a sharded scene must carry n_edges_global (distributed.shard_scene)")
        return ESFMLossFn.apply(Ps, pts3D, edges, vals, cam_ptr, pt_ptr, pt_perm, self.kernel_conf(), shard,
                                E_global)
