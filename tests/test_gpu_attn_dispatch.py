"""Parity of every size / occupancy dependent attention dispatch against the fp64 oracle (GPU).

gasfm_gat_attn_fwd picks its kernel from the problem (csrc/gat_attn.hip, "dispatch"):
  - attn_fwd_grp_kernel<U, MINW> (8 segments per wave task) for streamed 32-wide convs when the
    wave tasks fill >= GASFM_TUNE_ATTN_GRP_MIN_FILL (0.5) of the resident waves: the model's
    point direction (XL written in segment order by the prologue, xl_sorted) at >= ~16k points;
  - attn_fwd_glds_kernel (one item per wave, direct-to-LDS) for other streamed 32-wide convs;
  - attn_fwd_kernel / attn_fwd_generic otherwise; attn_fwd_lanes_kernel for block 0's 4-wide
    point direction (attention._lanes).
Each test records which kernel ran (gasfm_dispatch_counts) and asserts it, so a size change
cannot silently move a kernel out from under its parity test.

Reference semantics: PyG GATv2Conv as called at code/models/layers.py:426-432 (point
direction) and :329-335 (camera direction); oracle.pyg_gatv2.gatv2_segment_reference,
evaluated in fp64 (on the device at full config-4 size).
Tolerance (fp32 kernel vs fp64 oracle): |got - ref| <= 1e-5 + 1e-4 |ref| for
out / dXL / dXR; datt, dbias (sums over up to 4M edges) 1e-4 + 1e-4 |ref| normwise-scaled.
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from gasfm_amd import _native, synthetic
from gasfm_amd.attention import AttnPlan, attn_backward_raw, attn_forward_raw
from oracle.pyg_gatv2 import gatv2_segment_reference

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-5, 1e-4


def close(got, ref, atol=ATOL, rtol=RTOL, msg=""):
    torch.testing.assert_close(got.detach().double(), ref.detach().double().to(got.device), atol=atol, rtol=rtol,
                               msg=lambda m: f"{msg}: {m}")


def close_sum(got, ref, msg=""):
    """Reductions over all edges: elementwise within 1e-4 of the largest |ref| element."""
    got, ref = got.detach().double(), ref.detach().double().to(got.device)
    bound = 1e-4 * float(ref.abs().max()) + 1e-6
    err = float((got - ref).abs().max())
    assert err <= bound, f"{msg}: max |err| {err:.3e} > {bound:.3e}"


def seg_dst(plan):
    """Destination of each edge in segment order (row j of a segment-ordered XL)."""
    lens = (plan.seg_ptr[1:] - plan.seg_ptr[:-1]).long()
    return torch.repeat_interleave(torch.arange(plan.num_targets, device=lens.device), lens)


def oracle_sorted(XLs, XR, att, bias, plan, gout, H):
    """fp64 oracle forward + backward with XL in segment order: (out, max, sum, dXLs, dXR, datt, dbias)."""
    C = att.numel() // H
    d = lambda t: t.detach().double().requires_grad_(True)
    XLd, XRd, attd, biasd = d(XLs), d(XR), d(att.view(H, C)), d(bias)
    dst = seg_dst(plan).to(XLs.device)
    out, smax, ssum = gatv2_segment_reference(XLd.view(-1, H, C), XRd.view(-1, H, C), attd, biasd, dst,
                                              plan.num_targets)
    (out * gout.double()).sum().backward()
    return out, smax, ssum, XLd.grad, XRd.grad, attd.grad.reshape(-1), biasd.grad


def run_case(device, plan, XLs, XR, att, bias, H, gout, xl_sorted):
    """Kernel forward + backward; XLs is in segment order, the kernel gets it streamed (xl_sorted) or
    in edge order through perm.  Returns (results, forward counts, backward counts)."""
    if xl_sorted or plan.perm is None:
        XL_in = XLs
    else:
        XL_in = torch.empty_like(XLs)
        XL_in[plan.perm.long()] = XLs
    with _native.dispatch_record() as fr:
        out, smax, ssum = attn_forward_raw(XL_in, XR, att, bias, plan, H, 0.2, xl_sorted=xl_sorted)
        torch.cuda.synchronize()
    with _native.dispatch_record() as br:
        dXL, dXR, datt, dbias = attn_backward_raw(XL_in, XR, att, bias, plan, H, 0.2, out, smax, ssum, gout,
                                                  xl_sorted=xl_sorted)
        torch.cuda.synchronize()
    if plan.perm is not None:
        dXL = dXL[plan.perm.long()]  # edge order -> segment order
    return (out, smax, ssum, dXL, dXR, datt, dbias), fr.counts, br.counts


def compare(got, ref, nonempty, label):
    out, smax, ssum, dXL, dXR, datt, dbias = got
    r_out, r_max, r_sum, r_dXL, r_dXR, r_datt, r_dbias = ref
    close(out, r_out, msg=f"{label} out")
    close(smax[nonempty], r_max[nonempty], msg=f"{label} seg_max")
    close(ssum, r_sum, rtol=2e-4, msg=f"{label} seg_sum")
    close(dXL, r_dXL, msg=f"{label} dXL")
    close(dXR, r_dXR, atol=1e-4, msg=f"{label} dXR")
    close_sum(datt, r_datt, msg=f"{label} datt")
    close_sum(dbias, r_dbias, msg=f"{label} dbias")


def inputs(device, E, N, H, C, seed, xr_rows=None):
    g = torch.Generator(device=device).manual_seed(seed)
    XLs = torch.randn((E, H * C), generator=g, device=device)
    XR = torch.randn((N if xr_rows is None else xr_rows, H * C), generator=g, device=device)
    att = torch.randn((H * C,), generator=g, device=device) * (1.0 / C ** 0.5)  # non-zero attention
    bias = torch.randn((H * C,), generator=g, device=device)
    gout = torch.randn((N, H * C), generator=g, device=device)
    return XLs, XR, att, bias, gout


@pytest.fixture(scope="module")
def scene_plans(device):
    cache = {}

    def get(scale):
        if scale not in cache:
            sc = synthetic.config4() if scale == 1.0 else synthetic.scaled_config4(scale, seed=11)
            data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
            cache.clear()  # keep one config-4-size scene resident at a time
            cache[scale] = (sc, {k: w.plan for k, w in data.graph_wrappers.items()})
        return cache[scale]
    return get


@pytest.mark.parametrize("scale", [0.1, 1.0])
def test_point_direction_grouped_forward_vs_oracle(device, scene_plans, scale):
    """The model's point-direction conv exactly as the bench runs it (xl_sorted, no perm): the
    grouped-item forward must be the kernel that ran, at scaled_config4(0.1) (20k points, 2.5k wave
    tasks: the 2-groups-per-item form) and at full config 4 (200k points, 4,001,638 edges)."""
    sc, plans = scene_plans(scale)
    plan = plans["proj2scenepoint"]
    assert plan.perm is not None and plan.pos is not None
    H, C = 4, 8
    XLs, XR, att, bias, gout = inputs(device, plan.num_edges, plan.num_targets, H, C, seed=int(scale * 100))
    got, fwd, bwd = run_case(device, plan, XLs, XR, att, bias, H, gout, xl_sorted=True)
    assert fwd["attn_fwd_grp"] == 1 and sum(v for k, v in fwd.items() if not k.startswith("attn_fwd_grp_s")) == 1, fwd
    # 20k points (2.5k tasks of 8 items, under one round of resident waves): 2 lane groups per item;
    # config 4's 25k tasks: one group per item
    assert fwd["attn_fwd_grp_s2"] == (1 if scale < 1.0 else 0) and fwd["attn_fwd_grp_s4"] == 0, fwd
    assert bwd["attn_bwd_glds"] == 1, bwd
    ref = oracle_sorted(XLs, XR, att, bias, plan, gout, H)
    nonempty = (plan.seg_ptr[1:] > plan.seg_ptr[:-1]).to(device)
    compare(got, ref, nonempty, f"point scale {scale}")


@pytest.mark.parametrize("scale", [0.1, 1.0])
def test_camera_direction_split_items_vs_oracle(device, scene_plans, scale):
    """The camera direction (~4k-edge segments split into <= 256-edge pieces + ordered combines):
    the direct-to-LDS forward (too few items for the grouped kernel) with non-zero attention."""
    sc, plans = scene_plans(scale)
    plan = plans["proj2view"]
    assert plan.perm is None and plan.n_slots > 0
    H, C = 4, 8
    XLs, XR, att, bias, gout = inputs(device, plan.num_edges, plan.num_targets, H, C, seed=7 + int(scale * 100))
    got, fwd, bwd = run_case(device, plan, XLs, XR, att, bias, H, gout, xl_sorted=False)
    assert fwd["attn_fwd_glds"] == 1 and fwd["attn_fwd_grp"] == 0, fwd
    assert fwd["attn_combine_vec"] >= 1, fwd
    assert bwd["attn_bwd_glds"] == 1, bwd
    ref = oracle_sorted(XLs, XR, att, bias, plan, gout, H)
    nonempty = (plan.seg_ptr[1:] > plan.seg_ptr[:-1]).to(device)
    compare(got, ref, nonempty, f"camera scale {scale}")


def test_point_direction_gathered_vs_oracle(device, scene_plans):
    """The same point conv with XL in edge order read through perm (the PyG-call-form and sharded
    paths): the register kernel, since the streamed kernels need perm = NULL."""
    sc, plans = scene_plans(0.1)
    plan = plans["proj2scenepoint"]
    H, C = 4, 8
    XLs, XR, att, bias, gout = inputs(device, plan.num_edges, plan.num_targets, H, C, seed=5)
    got, fwd, bwd = run_case(device, plan, XLs, XR, att, bias, H, gout, xl_sorted=False)
    assert fwd["attn_fwd_vec"] == 1 and fwd["attn_fwd_grp"] == 0, fwd
    ref = oracle_sorted(XLs, XR, att, bias, plan, gout, H)
    nonempty = (plan.seg_ptr[1:] > plan.seg_ptr[:-1]).to(device)
    compare(got, ref, nonempty, "point gathered")


def random_sorted_plan(device, N, E, max_piece, seed, empty_frac=0.15):
    rng = np.random.default_rng(seed)
    w = rng.random(N) ** 3
    w[rng.random(N) < empty_frac] = 0
    w[0] = max(w[0], 1e-3)
    dst = np.sort(rng.choice(N, size=E, p=w / w.sum()))
    return AttnPlan.from_targets(torch.from_numpy(dst.astype(np.int64)), N, max_piece=max_piece).to(device)


# every variant of the forward dispatch, forced at a small size: (tuning, expected kernel)
VARIANTS = [
    (dict(attn_grp_rows=4, attn_grp_min_fill=0, attn_grp_split=1), "attn_fwd_grp"),
    # round 6: 2 / 4 lane groups per item (the small-shard form), states merged at the item's end
    (dict(attn_grp_rows=4, attn_grp_min_fill=0, attn_grp_split=2), "attn_fwd_grp_s2"),
    (dict(attn_grp_rows=4, attn_grp_min_fill=0, attn_grp_split=4), "attn_fwd_grp_s4"),
    (dict(attn_grp_rows=8, attn_grp_min_fill=0), "attn_fwd_grp"),
    (dict(attn_grp_rows=46, attn_grp_min_fill=0), "attn_fwd_grp"),
    (dict(attn_grp_rows=48, attn_grp_min_fill=0), "attn_fwd_grp"),
    (dict(attn_grp_rows=4, attn_grp_min_fill=1e9), "attn_fwd_glds"),
    (dict(attn_grp_rows=0, attn_glds=1), "attn_fwd_glds"),
    (dict(attn_grp_rows=0, attn_glds=0), "attn_fwd_vec"),
]


@pytest.mark.parametrize("tuning,kernel", VARIANTS)
@pytest.mark.parametrize("max_piece", [256, 7])
def test_forced_forward_variants_vs_oracle(device, tuning, kernel, max_piece):
    """Each forward kernel on one streamed 32-wide graph with empty, single-edge, long (split) and
    ragged segments; max_piece 7 makes most items partial (slot >= 0) + two-level combines."""
    N, E, H, C = 3000, 60000, 4, 8
    plan = random_sorted_plan(device, N, E, max_piece, seed=max_piece)
    XLs, XR, att, bias, gout = inputs(device, E, N, H, C, seed=3)
    with _native.tuned(**tuning):
        got, fwd, bwd = run_case(device, plan, XLs, XR, att, bias, H, gout, xl_sorted=False)
    # the split forms also count as attn_fwd_grp (one kernel launched)
    launched = sum(v for k, v in fwd.items() if k.startswith("attn_fwd") and not k.startswith("attn_fwd_grp_s"))
    assert fwd[kernel] == 1 and launched == 1, fwd
    if kernel.startswith("attn_fwd_grp"):
        assert fwd["attn_fwd_grp"] == 1 and fwd["attn_fwd_grp_s2"] == (kernel == "attn_fwd_grp_s2") \
            and fwd["attn_fwd_grp_s4"] == (kernel == "attn_fwd_grp_s4"), fwd
    ref = oracle_sorted(XLs, XR, att, bias, plan, gout, H)
    nonempty = (plan.seg_ptr[1:] > plan.seg_ptr[:-1]).to(device)
    compare(got, ref, nonempty, f"{kernel} {tuning}")


@pytest.mark.parametrize("tuning,kernel", [(dict(attn_glds=1), "attn_bwd_glds"),
                                           (dict(attn_glds=0), "attn_bwd_vec")])
@pytest.mark.parametrize("max_piece", [64, 7])
def test_forced_backward_variants_vs_oracle(device, tuning, kernel, max_piece):
    """Backward kernels of the 32-wide conv: direct-to-LDS and register, streamed and by position;
    max_piece 7: most items partial (dXR partial slots)."""
    N, E, H, C = 2000, 40000, 4, 8
    plan = random_sorted_plan(device, N, E, max_piece, seed=9)
    XLs, XR, att, bias, gout = inputs(device, E, N, H, C, seed=4)
    with _native.tuned(**tuning):
        got, fwd, bwd = run_case(device, plan, XLs, XR, att, bias, H, gout, xl_sorted=False)
    assert bwd[kernel] == 1, bwd
    ref = oracle_sorted(XLs, XR, att, bias, plan, gout, H)
    nonempty = (plan.seg_ptr[1:] > plan.seg_ptr[:-1]).to(device)
    compare(got, ref, nonempty, f"bwd {kernel} max_piece={max_piece}")


def test_lanes_rule_block0_point_direction(device, scene_plans):
    """Block 0's 4-wide point conv (H = 4, C = 1, ~20 edges per point): the lane-per-item forward
    (attention._lanes), streamed as the model passes it."""
    sc, plans = scene_plans(0.1)
    plan = plans["proj2scenepoint"]
    H, C = 4, 1
    XLs, XR, att, bias, gout = inputs(device, plan.num_edges, plan.num_targets, H, C, seed=12)
    got, fwd, bwd = run_case(device, plan, XLs, XR, att, bias, H, gout, xl_sorted=True)
    assert fwd["attn_fwd_lanes"] == 1, fwd
    ref = oracle_sorted(XLs, XR, att, bias, plan, gout, H)
    nonempty = (plan.seg_ptr[1:] > plan.seg_ptr[:-1]).to(device)
    compare(got, ref, nonempty, "block-0 lanes")


def test_three_block_model_scale01_dispatches_grouped_kernel(device):
    """A 3-block learning-conf net at scaled_config4(0.1) (200 cameras, 20k points, ~400k edges)
    against the functional fp64 oracle (oracle/gasfm_ref.py): outputs and every parameter
    gradient, with the grouped point forward and the lane-per-item block-0 forward recorded."""
    from conftest import check_grad, oracle_grads
    from oracle.weights import deterministic_state_dict
    sc = synthetic.scaled_config4(0.1, seed=11)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
    sd = deterministic_state_dict(net.state_dict(), torch.float64)
    net.load_state_dict({k: v.float() for k, v in sd.items()})
    net = net.to(device)
    gen = torch.Generator().manual_seed(3)
    cP = torch.randn((sc.m, 3, 4), generator=gen, dtype=torch.float64)
    cX = torch.randn((4, sc.n), generator=gen, dtype=torch.float64)
    with _native.dispatch_record() as rec:
        pred = net(data)
        ((pred["Ps_norm"] * cP.float().to(device)).sum() + (pred["pts3D"] * cX.float().to(device)).sum()).backward()
        torch.cuda.synchronize()
    # blocks 1, 2 and the final update: point direction grouped; block 0: lanes
    assert rec.counts["attn_fwd_grp"] == 3, rec.counts
    assert rec.counts["attn_fwd_lanes"] == 1, rec.counts
    (g64, r64), (g32, _) = oracle_grads(sd, sc, cP, cX)
    np.testing.assert_allclose(pred["Ps_norm"].detach().cpu().numpy(), r64["Ps_norm"].detach().numpy(),
                               atol=1e-4, rtol=1e-3)
    np.testing.assert_allclose(pred["pts3D"].detach().cpu().numpy(), r64["pts3D"].detach().numpy(),
                               atol=1e-4, rtol=1e-3)
    for k, p in net.named_parameters():
        check_grad(p.grad, g64[k], k, g32[k])
