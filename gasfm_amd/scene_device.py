"""Device-side scene graph construction.

The reference rebuilds every training sample's graph on the CPU, in DataLoader workers, from
the dense measurement matrix: ``get_M_valid_points`` / ``M2sparse`` / ``normalize_M``
(utils/dataset_utils.py:86-156, utils/geo_utils.py:689-703) and the four star graphs of
``SceneData.create_axial_aggregation_graphs`` (datasets/SceneData.py:153-239).  When M is
already in HBM, ``scene_from_dense_device`` builds the same ``SceneData`` on the GPU:

  edges, values, counts, point CSR   gasfm_scene_mask / _emit / _point_csr (csrc/scene_build.hip)
  work items of the attention plans  ``plan_work_device``: gasfm_plan_work (host_graph.cpp)
                                     restated over segment lengths with torch device ops
                                     (O(segments) glue, bit-identical items / slots / combines)

Everything the model reads is bit-identical to the host builder (``SceneData(M, Ns, ...)``):
edge order, indices, counts, plans; values agree to fp32 rounding of the 2x3 normalisation.
Host syncs: the edge count, the item counts of the four plans, and the small combine lists.
"""
import torch

from . import _native
from .attention import DEFAULT_MAX_PIECE, AttnPlan
from .scene import (MIN_N_POINTS_PER_VIEW, MIN_N_VIEWS_PER_POINT, AxialAggregationGraphWrapper, SceneData,
                    SparseMat)


def plan_work_device(seg_ptr, max_piece, all_partial=False):
    """gasfm_plan_work (host_graph.cpp) on device tensors: (items [I, 4], combine [K, 4], n_slots).

    Segment s of length len > max_piece splits into ceil(len / max_piece) pieces whose lengths
    differ by at most one (the first len % pieces are one longer); pieces take consecutive
    partial slots in segment order, from N when ``all_partial`` (then unsplit segments write
    slot s), else from 0 (unsplit: slot -1)."""
    ptr = seg_ptr.to(torch.int64)
    dev = ptr.device
    N = ptr.shape[0] - 1
    ln = ptr[1:] - ptr[:-1]
    split = ln > max_piece
    pieces = torch.where(split, (ln + max_piece - 1) // max_piece, torch.ones_like(ln))
    n_items = int(pieces.sum()) if N else 0
    seg = torch.repeat_interleave(torch.arange(N, device=dev), pieces, output_size=n_items)
    first = torch.cumsum(pieces, 0) - pieces
    p = torch.arange(n_items, device=dev) - first[seg]
    base, rem = ln // pieces, ln % pieces
    begin = ptr[:-1][seg] + p * base[seg] + torch.minimum(p, rem[seg])
    end = begin + base[seg] + (p < rem[seg]).to(torch.int64)
    sp = torch.where(split, pieces, torch.zeros_like(pieces))
    s0 = N if all_partial else 0
    slot_first = s0 + torch.cumsum(sp, 0) - sp
    unsplit = seg if all_partial else torch.full_like(seg, -1)
    slot = torch.where(split[seg], slot_first[seg] + p, unsplit)
    n_slots = s0 + (int(sp.sum()) if N else 0)
    cs = torch.nonzero(split).view(-1)
    combine = torch.stack([cs, slot_first[cs], pieces[cs], torch.ones_like(cs)], 1).to(torch.int32)
    items = torch.stack([seg, begin, end, slot], 1).to(torch.int32)
    return items.contiguous(), combine.contiguous(), n_slots


def _plan(seg_ptr, perm, pos, num_targets, num_edges, src_rows, max_piece, tag, all_partial=False):
    items, comb, n_slots = plan_work_device(seg_ptr, max_piece, all_partial)
    plan = AttnPlan(seg_ptr, perm, items, comb, n_slots, num_targets, num_edges, src_rows, all_partial, max_piece,
                    pos=pos)
    plan.tag = tag
    return plan


def _star_source_plan(src, src_rows, max_piece, tag):
    """One-target plan over source rows ``src`` (the global graphs): perm = src unless identity."""
    k = int(src.shape[0])
    dev = src.device
    seg_ptr = torch.tensor([0, k], dtype=torch.int32, device=dev)
    ident = k == 0 or bool(torch.equal(src, torch.arange(k, device=dev, dtype=src.dtype)))
    perm = None if ident else src.to(torch.int32).contiguous()
    return _plan(seg_ptr, perm, None, 1, k, src_rows, max_piece, tag)


def graph_wrappers_device(b, m, n, max_piece=None):
    """The four wrappers of build_graph_wrappers (scene.py) from ``_native.scene_build`` output."""
    mp = DEFAULT_MAX_PIECE if max_piece is None else max_piece
    cam, pt = b["cam"], b["pt"]
    E = int(cam.shape[0])
    indices = torch.stack([cam, pt])
    p2v = AxialAggregationGraphWrapper(m, n, 1, indices, build_plan=False)
    p2s = AxialAggregationGraphWrapper(m, n, 0, indices, build_plan=False)
    # camera direction: edges are cam-major already (seg_ptr = cam_ptr, no permutation)
    p2v.plan = _plan(b["cam_ptr"], None, None, m, E, E, mp, "proj2view")
    # point direction: the stable point CSR; a point-sorted edge list needs no permutation
    # (AttnPlan.from_targets takes its sorted branch then)
    sorted_pt = E <= 1 or bool((pt[1:] >= pt[:-1]).all())
    perm, pos = (None, None) if sorted_pt else (b["perm"], b["pos"])
    p2s.plan = _plan(b["pt_ptr"], perm, pos, n, E, E, mp, "proj2scenepoint")
    pts_per_cam = b["cam_ptr"][1:] - b["cam_ptr"][:-1]
    vv = torch.nonzero(pts_per_cam >= MIN_N_POINTS_PER_VIEW).view(-1)
    vp = torch.nonzero(b["pt_count"] >= MIN_N_VIEWS_PER_POINT).view(-1)
    v2g = AxialAggregationGraphWrapper(m, 1, 0, torch.stack([vv, torch.zeros_like(vv)]), build_plan=False)
    s2g = AxialAggregationGraphWrapper(1, n, 1, torch.stack([torch.zeros_like(vp), vp]), build_plan=False)
    v2g.plan = _star_source_plan(vv, m, 8, "view2global")
    s2g.plan = _star_source_plan(vp, n, min(256, max(16, -(-int(vp.shape[0]) // 4096))), "scenepoint2global")
    return {"proj2view": p2v, "proj2scenepoint": p2s, "view2global": v2g, "scenepoint2global": s2g}


def scene_from_dense_device(M, Ns, Ps_gt=None, scene_name="scene", calibrated=True, max_piece=None):
    """``SceneData(M, Ns, Ps_gt, scene_name)`` built on M's device (a CUDA tensor)."""
    m, n = M.shape[0] // 2, M.shape[1]
    b = _native.scene_build(M.contiguous(), Ns)
    cam_per_pts = b["pt_count"].to(torch.int64).unsqueeze(1)
    pts_per_cam = (b["cam_ptr"][1:] - b["cam_ptr"][:-1]).to(torch.int64).unsqueeze(1)
    self = SceneData.__new__(SceneData)
    self.scene_name = scene_name
    self.calibrated = calibrated
    self.y = Ps_gt
    self._M = M
    self.Ns = Ns
    self.device = M.device
    self.x = SparseMat(b["values"], torch.stack([b["cam"], b["pt"]]), cam_per_pts, pts_per_cam, (m, n, 2))
    self.graph_wrappers = graph_wrappers_device(b, m, n, max_piece)
    return self
