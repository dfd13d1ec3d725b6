"""Scene graph containers compatible with the reference's data path.

Mirrors the reference types the hot path consumes, with the same attribute
names and call signatures, so that ``GraphAttnSfMNet.forward(data)`` accepts
either the reference's own ``SceneData`` or this one:

  SparseMat                     utils/sparse_utils.py:392-449
  M2sparse / get_M_valid_points utils/dataset_utils.py:86-156
  AxialAggregationGraphWrapper  utils/dataset_utils.py:464-597
  SceneData (graph part)        datasets/SceneData.py:15-264

MI355X additions: every wrapper carries an ``AttnPlan`` (destination CSR,
point-direction permutation, balanced work items) built on the CPU when the
scene is built (DataLoader workers), and moved by ``.to(device)`` together
with the tensors the reference moves.
"""
import copy

import numpy as np
import torch

from .attention import AttnPlan

MIN_N_VIEWS_PER_POINT = 2   # utils/constants.py:2
MIN_N_POINTS_PER_VIEW = 8   # utils/constants.py:6


class SparseMat:
    """(m, n, F) sparse projection features: values [E, F], indices [2, E] (cam, pt)."""

    def __init__(self, values, indices, cam_per_pts, pts_per_cam, shape):
        assert len(shape) == 3
        self.values = values
        self.indices = indices
        self.shape = shape
        self.cam_per_pts = cam_per_pts
        self.pts_per_cam = pts_per_cam
        self.device = values.device

    @property
    def size(self):
        return self.shape

    def sum(self, dim):
        assert dim in (0, 1)
        out_size = self.shape[0] if dim == 1 else self.shape[1]
        idx = self.indices[0 if dim == 1 else 1]
        return torch.zeros(out_size, self.shape[2], device=self.device, dtype=self.values.dtype).index_add(
            0, idx, self.values)

    def mean(self, dim):
        return self.sum(dim) / (self.cam_per_pts if dim == 0 else self.pts_per_cam)

    def to(self, device, **kwargs):
        ret = copy.copy(self)
        ret.device = device
        ret.values = self.values.to(device, **kwargs)
        ret.indices = self.indices.to(device, **kwargs)
        ret.pts_per_cam = self.pts_per_cam.to(device, **kwargs)
        ret.cam_per_pts = self.cam_per_pts.to(device, **kwargs)
        return ret

    def __add__(self, other):
        assert self.shape == other.shape
        return SparseMat(self.values + other.values, self.indices, self.cam_per_pts, self.pts_per_cam, self.shape)

    def to_torch_hybrid_sparse_coo(self):
        return torch.sparse_coo_tensor(self.indices, self.values, size=self.shape).coalesce()


def get_M_valid_points(M):
    """(2m, n) or (m, n, 2) measurement matrix -> (m, n) validity mask (dataset_utils.py:86-113)."""
    if M.dim() == 2:
        M = M.reshape(-1, 2, M.shape[-1]).transpose(1, 2)
    valid = M.abs().sum(dim=2) != 0
    valid[:, valid.sum(dim=0) < MIN_N_VIEWS_PER_POINT] = False
    return valid


def M2sparse(M, normalize=False, Ns=None):
    """Dense (2m, n) M -> SparseMat (m, n, 2), cam-major edge order (dataset_utils.py:116-156)."""
    n_pts = M.shape[1]
    n_cams = M.shape[0] // 2
    valid = get_M_valid_points(M)
    cam_per_pts = valid.sum(dim=0).unsqueeze(1)
    pts_per_cam = valid.sum(dim=1).unsqueeze(1)
    idx = torch.from_numpy(np.array(np.nonzero(valid.cpu().numpy()))).to(M.device)
    M3 = M.reshape(n_cams, 2, n_pts).transpose(1, 2)
    if normalize:
        h = torch.cat([M3, torch.ones(n_cams, n_pts, 1, dtype=M.dtype, device=M.device)], dim=2)
        M3 = (h @ Ns.transpose(1, 2))[:, :, :2]
    vals = M3[idx[0], idx[1], :]
    return SparseMat(vals, idx, cam_per_pts, pts_per_cam, (n_cams, n_pts, 2))


class AxialAggregationGraphWrapper:
    """Row/column aggregation star graph (dataset_utils.py:464-597) plus its AttnPlan.

    ``edge_index``/``generate_node_features``/``extract_target_node_features`` keep the
    reference semantics (sources 0..E-1, targets E..E+N-1) so reference layer code can
    run on top of ``gasfm_amd.GATv2Conv``; ``plan`` is what the MI355X model uses.
    """

    def __init__(self, m, n, agg_dim, valid_indices, max_piece=None, build_plan=True):
        assert agg_dim in (0, 1)
        self.m, self.n = m, n
        self.agg_dim = agg_dim
        self.non_agg_dim = 1 - agg_dim
        self.n_agg_nodes = (m, n)[self.non_agg_dim]
        self.valid_indices = valid_indices
        self.device = valid_indices.device
        self.dense = False
        E = valid_indices.shape[1]
        self.edge_index = torch.stack([
            torch.arange(E, dtype=torch.int64, device=self.device),
            E + valid_indices[self.non_agg_dim]])
        self.plan = None
        if build_plan:
            kw = {} if max_piece is None else {"max_piece": max_piece}
            self.plan = AttnPlan.from_targets(valid_indices[self.non_agg_dim].cpu(), self.n_agg_nodes, **kw)

    def generate_node_features(self, M, x_agg=None):
        vals = M.values() if M.is_sparse else M.reshape(-1, M.shape[-1])
        if x_agg is None:
            x_agg = torch.zeros((self.n_agg_nodes, vals.shape[1]), dtype=vals.dtype, device=vals.device)
        return torch.cat((vals, x_agg), dim=0)

    def extract_target_node_features(self, x):
        if self.agg_dim == 0:
            return x[None, -self.n:, :]
        return x[-self.m:, None, :]

    def to(self, device, **kwargs):
        ret = copy.copy(self)
        ret.device = device
        ret.valid_indices = self.valid_indices.to(device, **kwargs)
        ret.edge_index = self.edge_index.to(device, **kwargs)
        if self.plan is not None:
            ret.plan = self.plan.to(device)
        return ret


def build_graph_wrappers(indices, m, n, max_piece=None, cam_max_piece=None):
    """The four aggregation graphs of SceneData.create_axial_aggregation_graphs (SceneData.py:153-239).
    cam_max_piece: the camera direction's work-item length when it differs from max_piece
    (attention.camera_max_piece for a point shard)."""
    cam, pt = indices[0], indices[1]
    dev = indices.device
    p2v = AxialAggregationGraphWrapper(m, n, 1, indices, max_piece if cam_max_piece is None else cam_max_piece)
    p2s = AxialAggregationGraphWrapper(m, n, 0, indices, max_piece)
    pts_per_cam = torch.bincount(cam, minlength=m)
    cam_per_pts = torch.bincount(pt, minlength=n)
    vv = torch.nonzero(pts_per_cam >= MIN_N_POINTS_PER_VIEW).view(-1)
    vp = torch.nonzero(cam_per_pts >= MIN_N_VIEWS_PER_POINT).view(-1)
    v2g = AxialAggregationGraphWrapper(m, 1, 0, torch.stack([vv, torch.zeros_like(vv)]).to(dev), build_plan=False)
    s2g = AxialAggregationGraphWrapper(1, n, 1, torch.stack([torch.zeros_like(vp), vp]).to(dev), build_plan=False)
    # global graphs: sources are view / point feature rows selected through the plan's perm
    v2g.plan = AttnPlan.from_targets(torch.zeros_like(vv), 1, src=vv, src_rows=m, max_piece=8)
    # ~4k pieces of >= 16 points: every wave streams a few 16-edge steps (a 256-edge piece is
    # 16 dependent load rounds, ~27 us whatever n is); the two-level combine merges the pieces
    s2g.plan = AttnPlan.from_targets(torch.zeros_like(vp), 1, src=vp, src_rows=n,
                                     max_piece=min(256, max(16, -(-vp.shape[0] // 4096))))
    out = {"proj2view": p2v, "proj2scenepoint": p2s, "view2global": v2g, "scenepoint2global": s2g}
    for name, w in out.items():
        w.plan.tag = name
    return out


class SceneData:
    """Graph-side subset of the reference SceneData (SceneData.py:15-264).

    Build from a dense measurement matrix (reference signature) or, for large
    synthetic scenes, with ``SceneData.from_sparse`` (no dense M).
    """

    def __init__(self, M, Ns, Ps_gt, scene_name, calibrated=True, max_piece=None):
        self.scene_name = scene_name
        self.calibrated = calibrated
        self.y = Ps_gt
        self._M = M
        self.Ns = Ns
        self.device = M.device
        self.x = M2sparse(M, normalize=True, Ns=Ns)
        self.graph_wrappers = build_graph_wrappers(self.x.indices, self.x.shape[0], self.x.shape[1], max_piece)

    @classmethod
    def from_sparse(cls, cam, pt, values, m, n, scene_name="synthetic", Ps_gt=None, max_piece=None,
                    cam_max_piece=None):
        self = cls.__new__(cls)
        self.scene_name = scene_name
        self.calibrated = True
        self.y = Ps_gt
        self._M = None
        self.Ns = None
        cam = torch.as_tensor(cam, dtype=torch.int64)
        pt = torch.as_tensor(pt, dtype=torch.int64)
        if cam.shape[0] > 1:
            key = cam * n + pt
            if not bool((key[1:] > key[:-1]).all()):
                raise ValueError("edges must be unique and cam-major sorted (M2sparse order)")
        indices = torch.stack([cam, pt])
        vals = torch.as_tensor(values, dtype=torch.float32)
        cam_per_pts = torch.bincount(pt, minlength=n).unsqueeze(1)
        pts_per_cam = torch.bincount(cam, minlength=m).unsqueeze(1)
        self.device = vals.device
        self.x = SparseMat(vals, indices, cam_per_pts, pts_per_cam, (m, n, vals.shape[1]))
        self.graph_wrappers = build_graph_wrappers(indices, m, n, max_piece, cam_max_piece)
        return self

    @classmethod
    def from_synthetic(cls, scene, max_piece=None):
        return cls.from_sparse(scene.cam, scene.pt, scene.normalized_values(), scene.m, scene.n,
                               scene_name="synthetic", Ps_gt=torch.from_numpy(scene.Ps_gt()), max_piece=max_piece)

    def __getattr__(self, name):
        # scenes built on the device (scene_device.scene_from_dense_device) build their four graph
        # wrappers on first use: the batched training path (batch.SceneBatch) reads the scene-build
        # arrays instead, and a scene that only feeds the loss never needs them
        if name == "graph_wrappers":
            lazy = self.__dict__.pop("_lazy_graph", None)
            if lazy is not None:
                self.graph_wrappers = lazy()
                return self.graph_wrappers
        raise AttributeError(name)

    def to(self, device, *args, dense_on_demand=False, **kwargs):
        if "_lazy_graph" in self.__dict__:
            self.graph_wrappers  # noqa: B018 (built before the copy: its closure holds this device's arrays)
        ret = copy.copy(self)
        ret.__dict__.pop("_scene_build", None)  # the copy reads its (moved) plans
        for key, attr in self.__dict__.items():
            if key.startswith("__") or key == "_scene_build" or (dense_on_demand and key in ("_M", "_norm_M")):
                continue
            if isinstance(attr, (SparseMat, AxialAggregationGraphWrapper)) or torch.is_tensor(attr):
                setattr(ret, key, attr.to(device, *args, **kwargs))
            elif isinstance(attr, dict):
                setattr(ret, key, {k: v.to(device, *args, **kwargs) for k, v in attr.items()})
        ret.device = device
        return ret
