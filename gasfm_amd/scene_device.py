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

Per-sample transforms before the build (§8(f) rank 3), with M staying on the device:
``sample_data_device`` (SceneData.sample_data) and ``apply_rotational_homography_aug_device``
(SceneData.apply_rotational_homography_aug, image points through gasfm_scene_homography); their
random draws come from the same numpy / torch CPU generators, in the reference's order.
"""
import math

import numpy as np
import torch

from . import _native
from .attention import DEFAULT_MAX_PIECE, L1_THRESHOLD, AttnPlan
from .scene import (MIN_N_POINTS_PER_VIEW, MIN_N_VIEWS_PER_POINT, AxialAggregationGraphWrapper, SceneData,
                    SparseMat)


def _piece_stats(ln, max_piece):
    """Per-segment piece counts of plan_work_device and the four host scalars it needs, on the device:
    (pieces, split, sp, scalars = [n_items, n_split, split pieces, level-1 combine entries])."""
    split = ln > max_piece
    pieces = torch.where(split, (ln + max_piece - 1) // max_piece, torch.ones_like(ln))
    sp = torch.where(split, pieces, torch.zeros_like(pieces))
    scalars = torch.stack([pieces.sum(), split.sum(), sp.sum(), _l1_groups(sp).sum()])
    return pieces, split, sp, scalars


def _l1_groups(cnt):
    """Level-1 entries of a combine over cnt slots (attention._two_level: groups of ceil(sqrt(cnt))
    when cnt > L1_THRESHOLD, else none); cnt = 0 gives 0."""
    g = torch.ceil(torch.sqrt(cnt.to(torch.float64))).to(torch.int64).clamp_(min=1)
    return torch.where(cnt > L1_THRESHOLD, (cnt + g - 1) // g, torch.zeros_like(cnt))


def _piece_counts_host(lengths, max_piece):
    """The scalars of _piece_stats for segment lengths known on the host (the one-segment global plans)."""
    n_items = n_split = n_sp = n_l1 = 0
    for ln in lengths:
        if ln > max_piece:
            pc = -(-ln // max_piece)
            n_items += pc
            n_split += 1
            n_sp += pc
            if pc > L1_THRESHOLD:
                g = int(math.ceil(math.sqrt(pc)))
                n_l1 += -(-pc // g)
        else:
            n_items += 1
    return [n_items, n_split, n_sp, n_l1]


def plan_work_device(seg_ptr, max_piece, all_partial=False, counts=None):
    """gasfm_plan_work (host_graph.cpp) on device tensors, with attention._two_level's split of the
    long combines: (items [I, 4], combine [K, 4], combine_l1 [K1, 4] or None, n_slots).

    Segment s of length len > max_piece splits into ceil(len / max_piece) pieces whose lengths
    differ by at most one (the first len % pieces are one longer); pieces take consecutive
    partial slots in segment order, from N when ``all_partial`` (then unsplit segments write
    slot s), else from 0 (unsplit: slot -1).  counts: the 4 host scalars of _piece_stats when the
    caller read them already (one host read per scene build instead of one per plan)."""
    ptr = seg_ptr.to(torch.int64)
    dev = ptr.device
    N = ptr.shape[0] - 1
    ln = ptr[1:] - ptr[:-1]
    pieces, split, sp, scalars = _piece_stats(ln, max_piece)
    if counts is None:
        counts = scalars.tolist() if N else [0, 0, 0, 0]
    n_items, n_split, n_sp, n_l1 = (int(v) for v in counts)
    seg = torch.repeat_interleave(torch.arange(N, device=dev), pieces, output_size=n_items)
    first = torch.cumsum(pieces, 0) - pieces
    p = torch.arange(n_items, device=dev) - first[seg]
    base, rem = ln // pieces, ln % pieces
    begin = ptr[:-1][seg] + p * base[seg] + torch.minimum(p, rem[seg])
    end = begin + base[seg] + (p < rem[seg]).to(torch.int64)
    s0 = N if all_partial else 0
    slot_first = s0 + torch.cumsum(sp, 0) - sp
    unsplit = seg if all_partial else torch.full_like(seg, -1)
    slot = torch.where(split[seg], slot_first[seg] + p, unsplit)
    n_slots = s0 + n_sp
    cs = torch.nonzero_static(split, size=n_split).view(-1)
    cnt, b = pieces[cs], slot_first[cs]
    items = torch.stack([seg, begin, end, slot], 1).to(torch.int32).contiguous()
    if n_l1 == 0:
        combine = torch.stack([cs, b, cnt, torch.ones_like(cs)], 1).to(torch.int32).contiguous()
        return items, combine, None, n_slots
    # two levels (attention._two_level): an entry over cnt > L1_THRESHOLD slots becomes ng level-1
    # entries over groups of g = ceil(sqrt(cnt)) slots (partial rows n_slots + k, in entry order)
    # and a level-2 entry over those rows
    ng = _l1_groups(cnt)
    g = torch.ceil(torch.sqrt(cnt.to(torch.float64))).to(torch.int64)
    first_l1 = n_slots + torch.cumsum(ng, 0) - ng
    e = torch.repeat_interleave(torch.arange(cs.shape[0], device=dev), ng, output_size=n_l1)
    k = torch.arange(n_l1, device=dev) - (torch.cumsum(ng, 0) - ng)[e]
    lo = b[e] + k * g[e]
    l1 = torch.stack([first_l1[e] + k, lo, torch.minimum(g[e], b[e] + cnt[e] - lo), torch.ones_like(e)], 1)
    big = ng > 0
    combine = torch.stack([cs, torch.where(big, first_l1, b), torch.where(big, ng, cnt), torch.ones_like(cs)], 1)
    return items, combine.to(torch.int32).contiguous(), l1.to(torch.int32).contiguous(), n_slots


def _plan(seg_ptr, perm, pos, num_targets, num_edges, src_rows, max_piece, tag, all_partial=False, counts=None):
    items, comb, comb_l1, n_slots = plan_work_device(seg_ptr, max_piece, all_partial, counts)
    plan = AttnPlan(seg_ptr, perm, items, comb, n_slots, num_targets, num_edges, src_rows, all_partial, max_piece,
                    pos=pos, combine_l1=comb_l1)
    plan.tag = tag
    return plan


def _star_source_plan(src, src_rows, max_piece, tag, ident=None):
    """One-target plan over source rows ``src`` (the global graphs): perm = src unless identity
    (ident: that test's answer when the caller read it already)."""
    k = int(src.shape[0])
    dev = src.device
    seg_ptr = torch.tensor([0, k], dtype=torch.int32, device=dev)
    if ident is None:
        ident = k == 0 or bool(torch.equal(src, torch.arange(k, device=dev, dtype=src.dtype)))
    perm = None if ident else src.to(torch.int32).contiguous()
    return _plan(seg_ptr, perm, None, 1, k, src_rows, max_piece, tag, counts=_piece_counts_host([k], max_piece))


def graph_wrappers_device(b, m, n, max_piece=None):
    """The four wrappers of build_graph_wrappers (scene.py) from ``_native.scene_build`` output.
    Every host scalar the four plans need (piece counts, valid view / point counts, sortedness)
    crosses to the host in ONE read."""
    mp = DEFAULT_MAX_PIECE if max_piece is None else max_piece
    cam, pt = b["cam"], b["pt"]
    E = int(cam.shape[0])
    indices = torch.stack([cam, pt])
    p2v = AxialAggregationGraphWrapper(m, n, 1, indices, build_plan=False)
    p2s = AxialAggregationGraphWrapper(m, n, 0, indices, build_plan=False)
    pts_per_cam = b["cam_ptr"][1:] - b["cam_ptr"][:-1]
    valid_v = pts_per_cam >= MIN_N_POINTS_PER_VIEW
    valid_p = b["pt_count"] >= MIN_N_VIEWS_PER_POINT
    ln_c = (b["cam_ptr"][1:] - b["cam_ptr"][:-1]).to(torch.int64)
    ln_p = (b["pt_ptr"][1:] - b["pt_ptr"][:-1]).to(torch.int64)
    sorted_pt = (pt[1:] >= pt[:-1]).all() if E > 1 else torch.ones((), dtype=torch.bool, device=cam.device)
    z = torch.zeros(4, dtype=torch.int64, device=cam.device)
    # valid ids == arange(k) <=> the valid flags are a prefix of ones
    vals = torch.cat([torch.stack([sorted_pt.to(torch.int64), valid_v.sum(), valid_p.sum(),
                                   (valid_v.to(torch.int64).cumprod(0).sum() if m else z[0]),
                                   (valid_p.to(torch.int64).cumprod(0).sum() if n else z[0])]),
                      _piece_stats(ln_c, mp)[3] if m else z, _piece_stats(ln_p, mp)[3] if n else z]).tolist()
    is_sorted, n_vv, n_vp, pre_v, pre_p = (int(v) for v in vals[:5])
    # camera direction: edges are cam-major already (seg_ptr = cam_ptr, no permutation)
    p2v.plan = _plan(b["cam_ptr"], None, None, m, E, E, mp, "proj2view", counts=vals[5:9])
    # point direction: the stable point CSR; a point-sorted edge list needs no permutation
    # (AttnPlan.from_targets takes its sorted branch then)
    perm, pos = (None, None) if is_sorted else (b["perm"], b["pos"])
    p2s.plan = _plan(b["pt_ptr"], perm, pos, n, E, E, mp, "proj2scenepoint", counts=vals[9:13])
    vv = torch.nonzero_static(valid_v, size=n_vv).view(-1)
    vp = torch.nonzero_static(valid_p, size=n_vp).view(-1)
    v2g = AxialAggregationGraphWrapper(m, 1, 0, torch.stack([vv, torch.zeros_like(vv)]), build_plan=False)
    s2g = AxialAggregationGraphWrapper(1, n, 1, torch.stack([torch.zeros_like(vp), vp]), build_plan=False)
    v2g.plan = _star_source_plan(vv, m, 8, "view2global", ident=pre_v == n_vv)
    s2g.plan = _star_source_plan(vp, n, min(256, max(16, -(-n_vp // 4096))), "scenepoint2global",
                                 ident=pre_p == n_vp)
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
    # the graph wrappers are built on first use (SceneData.__getattr__); batch.SceneBatch reads these
    self._scene_build = {k: b[k] for k in ("cam_ptr", "pt_ptr", "perm", "pos", "pt")}
    self._lazy_graph = lambda: graph_wrappers_device(b, m, n, max_piece)
    return self


# ------------------------------------------------------------------ per-sample transforms on the device
def _dense_M(data):
    M = getattr(data, "M", None)
    if M is None:
        M = getattr(data, "_M", None)
    if M is None:
        raise ValueError("the scene carries no dense measurement matrix M")
    return M


def sample_indices(N, num_samples, adjacent):
    """dataset_utils.sample_indices (utils/dataset_utils.py:25-40), same numpy RNG calls."""
    if num_samples == 1:
        return np.arange(N)
    if num_samples < 1:
        num_samples = int(np.ceil(num_samples * N))
    num_samples = max(2, num_samples)
    if num_samples >= N:
        return np.arange(N)
    if adjacent:
        start = np.random.randint(0, N - num_samples + 1)
        return np.arange(start, start + num_samples)
    return np.random.choice(N, num_samples, replace=False)


class DenseScene:
    """A sampled scene before its graph is built (``sample_data_device(..., build=False)``): the
    dense M with Ns / y, enough for ``apply_rotational_homography_aug_device`` (which builds the
    graph once, instead of once per transform)."""

    def __init__(self, M, Ns, y, scene_name, calibrated=True, host_Ns_y=None):
        self._M, self.Ns, self.y, self.scene_name, self.calibrated = M, Ns, y, scene_name, calibrated
        self.device = M.device
        self._host_Ns_y = host_Ns_y  # fp32 CPU copies of (Ns, y): the augmentation's 3x3 products


def sample_data_device(data, num_views, consecutive_views=True, max_piece=None, build=True):
    """SceneData.sample_data (datasets/SceneData.py:306-353) with M on the device: the view subset's
    rows, the points still seen in >= 2 of those views (gasfm_scene_mask's counts), then the
    device graph build (``build=False``: a DenseScene for a following transform that builds it).
    The view choice draws from numpy's global RNG exactly as the reference."""
    M = _dense_M(data)
    idx = sample_indices(len(data.y), num_views, adjacent=consecutive_views)
    m_idx = np.sort(np.concatenate((2 * idx, 2 * idx + 1)))
    dev = M.device
    ti = torch.from_numpy(idx).to(dev)
    y, Ns = data.y.to(dev)[ti], data.Ns.to(dev)[ti]
    Ms = M.index_select(0, torch.from_numpy(m_idx).to(dev)).contiguous()
    _, _, pt_count, _ = _native.scene_mask(Ms)
    keep = torch.nonzero(pt_count > 0).view(-1)  # get_M_valid_points(M).any(dim=0)
    Ms = Ms.index_select(1, keep).contiguous()
    if not build:
        # host copies of the full scene's Ns / y, read once per scene (not once per sample)
        hc = getattr(data, "_gasfm_host_Ns_y", None)
        if hc is None:
            hc = (data.Ns.float().cpu(), data.y.float().cpu())
            try:
                data._gasfm_host_Ns_y = hc
            except AttributeError:
                pass
        ih = torch.from_numpy(idx)
        return DenseScene(Ms, Ns.contiguous(), y, data.scene_name, getattr(data, "calibrated", True),
                          host_Ns_y=(hc[0][ih], hc[1][ih]))
    return scene_from_dense_device(Ms, Ns.contiguous(), y, data.scene_name,
                                   calibrated=getattr(data, "calibrated", True), max_piece=max_piece)


def _axis_angle_to_matrix(axis_angle):
    """pytorch3d.transforms.axis_angle_to_matrix (published formula: axis-angle -> quaternion with
    the small-angle series below 1e-6 -> quaternion_to_matrix, real part first)."""
    angles = torch.norm(axis_angle, p=2, dim=-1, keepdim=True)
    half = angles * 0.5
    small = angles.abs() < 1e-6
    safe = torch.where(small, torch.ones_like(angles), angles)
    s = torch.where(small, 0.5 - angles * angles / 48, torch.sin(half) / safe)
    q = torch.cat([torch.cos(half), axis_angle * s], dim=-1)
    r, i, j, k = torch.unbind(q, -1)
    two_s = 2.0 / (q * q).sum(-1)
    o = torch.stack((1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                     two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                     two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)), -1)
    return o.reshape(q.shape[:-1] + (3, 3))


def rotational_homography(num_views, inplane_rot_aug_max_angle=None, tilt_rot_aug_max_angle=None):
    """R_aug [m, 3, 3] of SceneData.apply_rotational_homography_aug (SceneData.py:373-406), drawn from
    torch's global CPU RNG in the reference's order (in-plane angle, tilt angle, tilt axis)."""
    R = torch.eye(3)[None, :, :].repeat(num_views, 1, 1)
    inplane = inplane_rot_aug_max_angle or 0
    tilt = tilt_rot_aug_max_angle or 0
    assert inplane >= 0 and tilt >= 0
    if inplane > 0:
        ang = inplane * (2 * torch.rand((num_views,), dtype=torch.float32) - 1)
        vec = torch.zeros((num_views, 3), dtype=torch.float32)
        vec[:, 2] = ang / 180. * math.pi
        R = _axis_angle_to_matrix(vec) @ R
    if tilt > 0:
        ang = tilt * (2 * torch.rand((num_views,), dtype=torch.float32) - 1)
        alpha = torch.rand((num_views,), dtype=torch.float32) * 2 * math.pi
        axis = torch.zeros((num_views, 3), dtype=torch.float32)
        axis[:, 0] = torch.cos(alpha)
        axis[:, 1] = torch.sin(alpha)
        R = _axis_angle_to_matrix(axis * ang[:, None] / 180. * math.pi) @ R
    return R


def apply_rotational_homography_aug_device(data, inplane_rot_aug_max_angle=None, tilt_rot_aug_max_angle=None,
                                           max_piece=None):
    """SceneData.apply_rotational_homography_aug (datasets/SceneData.py:355-440) with M on the device:
    the per-camera 3x3 products (R_aug, H_aug = Ns^-1 R_aug Ns, y' = H_aug y) on the host in fp32
    as the reference computes them, the image points through gasfm_scene_homography, then the
    device graph build."""
    M = _dense_M(data)
    m = data.y.shape[0]
    dev = M.device
    hc = getattr(data, "_host_Ns_y", None)
    Ns_c, y_c = hc if hc is not None else (data.Ns.float().cpu(), data.y.float().cpu())
    if not (inplane_rot_aug_max_angle or tilt_rot_aug_max_angle):
        return scene_from_dense_device(M, data.Ns.to(dev), data.y.to(dev), data.scene_name, max_piece=max_piece)
    R = rotational_homography(m, inplane_rot_aug_max_angle, tilt_rot_aug_max_angle)
    Ninv = torch.linalg.inv(Ns_c)
    y = (Ninv @ R @ Ns_c) @ y_c
    Mn = _native.scene_homography(M.contiguous(), Ns_c.to(dev).contiguous(), R.to(dev).contiguous(),
                                  Ninv.to(dev).contiguous())
    return scene_from_dense_device(Mn, Ns_c.to(dev), y.to(dev), data.scene_name,
                                   calibrated=getattr(data, "calibrated", True), max_piece=max_piece)
