"""Autograd wrappers of the fused per-edge block kernels (gasfm_amd/csrc/edge_block.hip).

A GASFM block (layers.py:222-263) on its E projection rows is expressed with
three differentiable ops whose forward AND backward are HIP kernels:

  EdgePrologueFn   P -> (XL = [Wl_pt; Wl_cam] relu(LN(P)) + b,  token)
  DualAttentionFn  XL -> (point aggregates, camera aggregates)   (fused GATv2 kernels)
  EdgeEpilogueFn   (P, P0, token, Sp, Sv, Sg) -> P' = P + (Wp [P_hat|P0] + bp + Sp[pt] + Sv[cam] + Sg)/4

P_hat = relu(LN(P)) is never materialised: both kernels recompute it from P.
The `token` output of the prologue is a zero-stride placeholder (its one element is never
read: an uninitialised 1x1 tensor, no fill kernel) whose gradient
the epilogue's backward sets to dP' (the block-output gradient), so that the
prologue's backward kernel can do the whole P-side backward in one pass:
  dP = LN_bwd(mask * (Wl^T dXL + Wp^T dP'/4)) + dP'      (identity residual, layers.py:254-261)
For the 32-wide blocks the prologue and the camera-direction attention are one kernel
(EdgeCamFn, csrc/edge_cam.hip).  Node-level work between them runs in the fused point /
view / global kernels (point_block.py, view_block.py, dense.py: csrc/point_block.hip,
view_block.hip, global_vec.hip); only the camera side's two m x 1024 x 1024 GEMMs per block
go through hipBLASLt (or the HIP MFMA GEMMs, view_block._mm).
"""
import os

import torch

from . import _native
from .attention import (attn_backward_raw, attn_forward_partial, attn_forward_raw, bwd_combine, bwd_combine2,
                        combine_fwd_l1, combine_partials)

PROJ_SCALE = 0.25  # the "/ 4" of layers.py:945
# EdgeCamFn's backward as ONE kernel (gasfm_edge_cam_pbwd: camera attention backward + edge
# prologue backward, dXLc never stored); 0 selects the two kernels edge_cam_bwd + edge_prologue_bwd
CAM_PBWD = os.environ.get("GASFM_CAM_PBWD", "1") != "0"
# The edge epilogue's backward folded into edge_cam_pbwd (round 3): block b's lin_proj weight
# gradient in block b's own edge_cam_pbwd (it holds dRes = dP' and relu(LN_b(P_b))), dSv / dP0 in
# block b+1's (the kernel that produces dP').  0: edge_epilogue_bwd as before.
EPI_FOLD = os.environ.get("GASFM_EPI_FOLD", "1") != "0"
# Measured and removed in round 5 (kept in git history): dXLp in point-segment order
# (GASFM_DXL_PT), block 0's epilogue backward folded into block 1's edge_cam_pbwd (GASFM_E0_FOLD),
# XLc kept by the forward seam instead of recomputed (GASFM_XLC_STORE).

# Block 0's prologue writes XL0 row by row through the point plan's permutation (one 32-B store
# per row, gasfm_edge0_prologue_fwd_rows) instead of scattering the point halves through pos.
E0_ROWS = os.environ.get("GASFM_E0_ROWS", "1") != "0"


def _rows(t):
    """Row block with unit column stride (a column slice of a gathered [SV | XR] block stays a view)."""
    return t if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1] else t.contiguous()


class EdgePrologueFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, P, ln_w, ln_b, W, b, Wp, eps, pos=None, W2=None, b2=None):
        """XL = [W; W2] relu(LN(P)) + [b; b2]: W2/b2 given, W/b and W2/b2 are the point- and
        camera-direction lin_l (each 32 x 32) as they are, else W [64 x 32] holds both.
        pos (point plan's inverse permutation): write the point half of XL in point order."""
        E = P.shape[0]
        XL = torch.empty((E, 64), dtype=torch.float32, device=P.device)
        split = W2 is not None
        _native.edge_prologue_fwd(P, ln_w, ln_b, eps, W.contiguous(), b.contiguous(), XL, pos,
                                  W2.contiguous() if split else None, b2.contiguous() if split else None)
        ctx.eps = eps
        ctx.has_ln = ln_w is not None
        ctx.split = split
        ctx.defer = _native.defer_token(ln_w, ln_b, W, b, W2, b2)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(P, ln_w, ln_b, W, Wp, W2)
        token = P.new_empty((1, 1)).expand(E, P.shape[1])
        return XL, token

    @staticmethod
    def backward(ctx, dXL, dtoken):
        P, ln_w, ln_b, W, Wp, W2 = ctx.saved_tensors
        E = P.shape[0]
        if dXL is None:
            dXL = torch.zeros((E, 64), dtype=torch.float32, device=P.device)
        dXL = dXL.contiguous()
        dRes = None
        if dtoken is not None and dtoken.stride(0) != 0:
            dRes = dtoken.contiguous()
        dP = torch.empty_like(P)
        rows = _native.edge_part_floats(0, E) // (64 * 32 + 64 + 64)
        part = torch.empty((rows, 64 * 32 + 64 + 64), dtype=torch.float32, device=P.device)
        _native.edge_prologue_bwd(dXL, P, dRes, ln_w, ln_b, ctx.eps, W.contiguous(),
                                  Wp.contiguous() if dRes is not None else None, PROJ_SCALE, dP, part,
                                  W2.contiguous() if W2 is not None else None)
        tot = _native.param_colsum(part.view(rows, -1), ctx.defer)
        dW = tot[:64 * 32].view(64, 32)
        db = tot[64 * 32:64 * 32 + 64]
        dgam = tot[64 * 32 + 64:64 * 32 + 96] if ctx.has_ln else None
        dbet = tot[64 * 32 + 96:] if ctx.has_ln else None
        if ctx.split:
            return dP, dgam, dbet, dW[:32], db[:32], None, None, None, dW[32:], db[32:]
        return dP, dgam, dbet, dW, db, None, None, None, None, None


def _cam_attention_fwd(launch, bias, plan, heads, HC, plan_partial, shard, dev):
    """Run a camera-item kernel (launch(items, n_items, finalize, out, smax, ssum, part)) and finish
    the camera attention: split pieces combined (one GPU), or the rank's partial rows all-gathered
    and merged in rank order (point-sharded).  Returns (out, seg_max, seg_sum)."""
    N = plan.num_targets
    LDP = HC + 2 * heads
    if shard is None:
        out = torch.empty((N, HC), dtype=torch.float32, device=dev)
        smax = torch.empty((N, heads), dtype=torch.float32, device=dev)
        ssum = torch.empty((N, heads), dtype=torch.float32, device=dev)
        part = torch.empty((plan.n_part_rows, LDP), dtype=torch.float32, device=dev) if plan.n_slots else None
        launch(plan.items, plan.n_items, True, out, smax, ssum, part)
        combine_fwd_l1(plan, part, heads, HC // heads)
        if plan.n_combine:
            _native.attn_combine(plan.combine, plan.n_combine, heads, HC // heads, part, bias, True, out, smax, ssum)
        return out, smax, ssum
    # local partial rows (attention.attn_forward_partial) -> all-gather -> ordered combine
    pp = plan_partial
    part = torch.empty((max(pp.n_part_rows, N), LDP), dtype=torch.float32, device=dev)
    if pp.n_items:
        launch(pp.items, pp.n_items, False, None, None, None, part)
        combine_fwd_l1(pp, part, heads, HC // heads)
        if pp.n_combine:
            _native.attn_combine(pp.combine, pp.n_combine, heads, HC // heads, part, None, False, part,
                                 part[:, HC:], part[:, HC + heads:], ldOut=LDP, ldStat=LDP)
    else:
        part[:N, :HC] = 0.0
        part[:N, HC:HC + heads] = -float("inf")
        part[:N, HC + heads:] = 0.0
    gathered = shard.all_gather(part[:N])
    return combine_partials(gathered, shard.world, N, heads, bias, shard.combine_items(N, dev))


class EdgeCamFn(torch.autograd.Function):
    """EdgePrologueFn + the camera half of DualAttentionFn in one pass (csrc/edge_cam.hip):

        P -> (XLp [E, 32] = Wpt relu(LN(P)) + bpt  (point order when pos is given),
              camera aggregates out_c [m, 32],
              token)

    XLc = Wc relu(LN(P)) + bc, the camera conv's lin_l rows, lives only in registers: the
    backward recomputes it from P.  token: as EdgePrologueFn's (its gradient is the block
    output's gradient dP', which the backward folds into dP with Wp).  plan_cam_partial / shard:
    point-sharded execution (camera segments span ranks: local partial rows, all-gather, ordered
    combine), as DualAttentionFn."""

    @staticmethod
    def forward(ctx, P, ln_w, ln_b, Wpt, bpt, Wc, bc, Wp, eps, pos, XR, att, bias, plan, heads, slope,
                plan_partial=None, shard=None, P0=None, dwp=False):
        """dwp: the backward also returns Wp's gradient, the block's edge-epilogue weight gradient
        scale sum_e dP'[e]^T [relu(LN(P[e])) | P0[e]] (dP' = the token's gradient), which the
        epilogue then leaves out (EdgeEpilogueFn's wp_by_cam)."""
        E, dev = P.shape[0], P.device
        HC = att.numel()
        if heads != 4 or HC != 32:
            raise ValueError("EdgeCamFn: the fused kernels are for H = 4, C = 8")
        attf = att.reshape(-1).contiguous()
        XLp = torch.empty((E, 32), dtype=torch.float32, device=dev)

        def launch(items, n_items, finalize, out, smax, ssum, part):
            _native.edge_cam_fwd(P, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, pos, XR, attf, bias if finalize else None,
                                 slope, items, n_items, finalize, out, smax, ssum, part)
        out, smax, ssum = _cam_attention_fwd(launch, bias, plan, heads, HC, plan_partial, shard, dev)
        ctx.eps, ctx.heads, ctx.slope, ctx.plan = eps, heads, slope, plan
        ctx.att_shape = att.shape
        ctx.has_ln = ln_w is not None
        ctx.dwp = bool(dwp)
        ctx.sharded = shard is not None
        ctx.defer = _native.defer_token(ln_w, ln_b, Wpt, bpt, Wc, bc, att, bias, Wp if dwp else None)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(P, ln_w, ln_b, Wpt, Wc, bc, Wp, XR, attf, bias, out, smax, ssum, P0)
        token = P.new_empty((1, 1)).expand(E, P.shape[1])
        return XLp, out, token

    @staticmethod
    def backward(ctx, dXLp, g_c, dtoken):
        dRes = dtoken.contiguous() if (dtoken is not None and dtoken.stride(0) != 0) else None
        return _cam_backward(ctx, ctx.saved_tensors, dXLp, g_c, dRes)


def _dwp_torch(P, ln_w, ln_b, eps, dRes, P0):
    """The epilogue weight gradient scale dRes^T [relu(LN(P)) | P0] with torch ops (the EdgeCamFn
    backward paths without edge_cam_pbwd)."""
    ph = torch.relu(torch.nn.functional.layer_norm(P, (P.shape[1],), ln_w, ln_b, eps))
    if P0 is not None:
        ph = torch.cat([ph, P0], dim=1)
    return PROJ_SCALE * (dRes.t() @ ph)


def _cam_backward(ctx, saved, dXLp, g_c, dRes, epi=None, dXR=None):
    """EdgeCamFn's backward from its saved state (ctx attributes eps, heads, slope, plan, att_shape,
    has_ln, dwp, defer): the 20 input gradients of EdgeCamFn.forward.  epi: the previous block's
    epilogue outputs to fill from dP (edge_cam_pbwd's EPI), or None; ctx.epi_done tells whether
    they were filled.  dXR: the [num_targets, 32] buffer for the camera target rows' gradient (a
    view of the boundary all-reduce's payload, _boundary_buffers), or None."""
    P, ln_w, ln_b, Wpt, Wc, bc, Wp, XR, attf, bias, out, smax, ssum, P0 = saved
    plan = ctx.plan
    E, dev = P.shape[0], P.device
    dXLp = torch.zeros((E, 32), dtype=torch.float32, device=dev) if dXLp is None else dXLp.contiguous()
    g_c = torch.zeros_like(out) if g_c is None else (g_c if g_c.stride(1) == 1 else g_c.contiguous())
    dwp = ctx.dwp and dRes is not None and ln_w is not None
    ctx.epi_done = False
    dWp = None
    if CAM_PBWD and plan.n_items:
        # camera attention backward + prologue backward in one kernel (gasfm_edge_cam_pbwd)
        if dXR is None:
            dXR = torch.empty((plan.num_targets, 32), dtype=torch.float32, device=dev)
        part_dxr = torch.empty((plan.n_part_rows, 32), dtype=torch.float32, device=dev) if plan.n_slots else None
        wcols = (34 if P0 is not None else 32) if dwp else 0
        rows, cols = _native.edge_cam_pbwd_part_shape(plan.n_items, wcols)
        part = torch.empty((rows, cols), dtype=torch.float32, device=dev)
        dP = torch.empty_like(P)
        use_epi = epi is not None and (ln_w is None) == (dRes is None)
        _native.edge_cam_pbwd(P, ln_w, ln_b, ctx.eps, Wpt.contiguous(), Wc.contiguous(), bc.contiguous(),
                              Wp.contiguous() if dRes is not None else None, PROJ_SCALE, XR, attf, bias, ctx.slope,
                              out, smax, ssum, g_c, plan.items, plan.n_items, dXLp, dRes, dP, dXR, part_dxr, part,
                              epi=epi if use_epi else None,
                              dwp=(P0 if P0 is not None else True) if dwp else None)
        ctx.epi_done = use_epi
        ctx.epi_combined = False
        if use_epi and part_dxr is not None and epi[3] is not None:
            # the split cameras' dXR and (EPI) dSv rows share their slots: one combine launch
            bwd_combine2(plan, part_dxr, dXR, epi[3], epi[2], 32)
            ctx.epi_combined = True
        else:
            bwd_combine(plan, part_dxr, 32, dXR)
        tot = _native.param_colsum(part, ctx.defer)
        o = 64 * 32
        ta = tot[o + 128:o + 192]
        if dwp:
            dWp = tot[o + 192:o + 192 + 32 * wcols].view(32, wcols)
    else:
        # camera attention backward (XLc recomputed from P): dXLc, dXR, [datt | dbias] partials
        dXLc = torch.empty((E, 32), dtype=torch.float32, device=dev)
        if dXR is None:
            dXR = torch.empty((plan.num_targets, 32), dtype=torch.float32, device=dev)
        part_dxr = torch.empty((plan.n_part_rows, 32), dtype=torch.float32, device=dev) if plan.n_slots else None
        rows, cols = _native.edge_cam_bwd_part_shape(plan.n_items)
        part_a = (torch.empty if plan.n_items else torch.zeros)((rows, cols), dtype=torch.float32, device=dev)
        if plan.n_items:
            _native.edge_cam_bwd(P, ln_w, ln_b, ctx.eps, Wc.contiguous(), bc.contiguous(), XR, attf, bias, ctx.slope,
                                 out, smax, ssum, g_c, plan.items, plan.n_items, dXLc, dXR, part_dxr, part_a)
            bwd_combine(plan, part_dxr, 32, dXR)
        else:  # no local edges
            dXLc.zero_()
            dXR.zero_()
        # prologue backward on [dXLp | dXLc] (+ the block output's residual gradient)
        dP = torch.empty_like(P)
        prow = _native.edge_part_floats(0, E) // (64 * 32 + 64 + 64)
        part = torch.empty((prow, 64 * 32 + 64 + 64), dtype=torch.float32, device=dev)
        _native.edge_prologue_bwd(dXLp, P, dRes, ln_w, ln_b, ctx.eps, Wpt.contiguous(),
                                  Wp.contiguous() if dRes is not None else None, PROJ_SCALE, dP, part, Wc.contiguous(),
                                  dXLc=dXLc)
        ta = _native.param_colsum(part_a, ctx.defer)
        tot = _native.param_colsum(part, ctx.defer)
        o = 64 * 32
        if dwp:
            dWp = _dwp_torch(P, ln_w, ln_b, ctx.eps, dRes, P0) if plan.n_items else torch.zeros_like(Wp)
    if dwp and dWp is None:  # no local edges
        dWp = torch.zeros_like(Wp)
    dW, db = tot[:o].view(64, 32), tot[o:o + 64]
    dgam = tot[o + 64:o + 96] if ctx.has_ln else None
    dbet = tot[o + 96:o + 128] if ctx.has_ln else None
    dbias = ta[32:]
    if getattr(ctx, "sharded", False) or (CAM_PBWD and plan.n_items):
        # edge_cam_pbwd leaves the bias gradient to this column sum of gout over all targets
        dbias = replicated_dbias(g_c, ctx.defer)
    return (dP, dgam, dbet, dW[:32], db[:32], dW[32:], db[32:], dWp, None, None, dXR,
            ta[:32].view(ctx.att_shape), dbias, None, None, None, None, None, None, None)


def replicated_dbias(gout, defer):
    """The attention bias gradient of a conv whose targets are replicated over point shards (the
    camera direction): the column sum of the replicated output gradient over ALL targets, so every
    rank gets the same bits.  The kernels' own d bias sums gout over the rank's local work items
    (first item of each segment), whose split and order differ between ranks (round 5: caught by
    the world-8 test, tests/test_distributed.py).  Deferred into the end-of-backward batched sums."""
    g = gout.reshape(gout.shape[0], int(gout[0].numel()) if gout.shape[0] else gout.shape[-1])
    if not (g.stride(1) == 1 and g.stride(0) >= g.shape[1]):  # e.g. an expanded (stride-0) gradient
        g = g.contiguous()
    # a view, as every other deferred sum reaches AccumulateGrad: the sum tensor itself is also held
    # by the pending job list, so AccumulateGrad would copy it (unfilled) instead of adopting it
    return _native.param_colsum(g, defer)[:]


class DualAttentionFn(torch.autograd.Function):
    """Point- and camera-direction GATv2 attention over the two halves of XL [E, 64].

    xl_sorted: the point half of XL is stored in point-segment order (EdgePrologueFn with
    pos); its gradient is still returned in edge order."""

    @staticmethod
    def forward(ctx, XL, XR_pt, XR_cam, att_pt, att_cam, bias_pt, bias_cam, plan_pt, plan_cam, heads, slope,
                plan_cam_partial=None, shard=None, xl_sorted=False):
        h = XL.shape[1] // 2
        XLp, XLc = XL[:, :h], XL[:, h:]
        out_p, mp, sp = attn_forward_raw(XLp, XR_pt, att_pt, bias_pt, plan_pt, heads, slope, xl_sorted=xl_sorted)
        if shard is None:
            out_c, mc, sc = attn_forward_raw(XLc, XR_cam, att_cam, bias_cam, plan_cam, heads, slope)
        else:  # camera segments span ranks: local partials -> all-gather -> ordered combine
            part = attn_forward_partial(XLc, XR_cam, att_cam, plan_cam_partial, heads, slope)
            gathered = shard.all_gather(part)
            N = plan_cam.num_targets
            out_c, mc, sc = combine_partials(gathered, shard.world, N, heads, bias_cam,
                                             shard.combine_items(N, XL.device))
        ctx.plans = (plan_pt, plan_cam)
        ctx.heads, ctx.slope, ctx.xl_sorted = heads, slope, xl_sorted
        ctx.sharded = shard is not None
        ctx.defer = _native.defer_token(att_pt, att_cam, bias_pt, bias_cam)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(XL, XR_pt, XR_cam, att_pt, att_cam, bias_pt, bias_cam, out_p, mp, sp, out_c, mc, sc)
        return out_p, out_c

    @staticmethod
    def backward(ctx, g_p, g_c):
        XL, XR_pt, XR_cam, att_pt, att_cam, bias_pt, bias_cam, out_p, mp, sp, out_c, mc, sc = ctx.saved_tensors
        plan_pt, plan_cam = ctx.plans
        h = XL.shape[1] // 2
        if g_p is None:
            g_p = torch.zeros_like(out_p)
        if g_c is None:
            g_c = torch.zeros_like(out_c)
        dXL = torch.empty_like(XL)
        _, dXRp, dattp, dbp = attn_backward_raw(XL[:, :h], XR_pt, att_pt, bias_pt, plan_pt, ctx.heads, ctx.slope,
                                                out_p, mp, sp, g_p, dXL=dXL[:, :h], xl_sorted=ctx.xl_sorted,
                                                defer=ctx.defer)
        _, dXRc, dattc, dbc = attn_backward_raw(XL[:, h:], XR_cam, att_cam, bias_cam, plan_cam, ctx.heads, ctx.slope,
                                                out_c, mc, sc, g_c, dXL=dXL[:, h:], defer=ctx.defer)
        if ctx.sharded:
            dbc = replicated_dbias(g_c, ctx.defer)
        return (dXL, dXRp, dXRc, dattp.view_as(att_pt), dattc.view_as(att_cam), dbp, dbc, None, None, None, None,
                None, None, None)


class EdgeEpilogueFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, P, P0, token, Sp, Sv, Sg, Wp, bp, ln_w, ln_b, eps, edges, wp_by_cam=False):
        """wp_by_cam: Wp's gradient is returned by the block's EdgeCamFn / SeamFn (its dwp), not here."""
        out = torch.empty_like(P)
        Wp_c = Wp.contiguous()
        _native.edge_epilogue_fwd(P, P0, edges.cam, edges.pt, ln_w, ln_b, eps, Wp_c, bp.contiguous(),
                                  Sp.contiguous(), _rows(Sv), Sg.reshape(-1).contiguous(), PROJ_SCALE, out)
        ctx.eps = eps
        ctx.edges = edges
        ctx.sg_shape = Sg.shape
        ctx.wp_by_cam = bool(wp_by_cam)
        ctx.defer = _native.defer_token(Wp)
        ctx.defer_b = _native.defer_token(bp)
        ctx.save_for_backward(P, P0, Wp_c, ln_w, ln_b)
        return out

    @staticmethod
    def backward(ctx, dPo):
        return _epilogue_backward(ctx, ctx.saved_tensors, dPo)


def _epilogue_backward(ctx, saved, dPo, folded=None, dSg=None):
    """EdgeEpilogueFn's backward from its saved state (ctx attributes eps, edges, sg_shape,
    wp_by_cam, defer, defer_b): the 13 input gradients of EdgeEpilogueFn.forward (the block input's
    through the token).  folded: (dSv, part_dsv, dP0) already filled by the next block's
    edge_cam_pbwd (SeamFn), so edge_epilogue_bwd does not run (Wp's gradient is then the block's
    EdgeCamFn's).  dSg: its [32] destination (a view of the boundary all-reduce's payload) or None."""
    P, P0, Wp, ln_w, ln_b = saved
    edges = ctx.edges
    dPo = dPo.contiguous()
    dev = P.device
    pc = edges.plans["proj2view"]
    pp = edges.plans["proj2scenepoint"]
    dWp = None
    if folded is not None:  # part_dsv None: merged together with the camera plan's dXR (edge_cam_pbwd)
        dSv, part_dsv, dP0 = folded
    else:
        # camera side: dSv (+ dWp, dP0) in one pass over the camera work items
        dSv = torch.empty((edges.m, 32), dtype=torch.float32, device=dev)
        part_dsv = torch.empty((max(pc.n_part_rows, 1), 32), dtype=torch.float32, device=dev)
        dP0 = torch.empty((P.shape[0], 2), dtype=torch.float32, device=dev) if P0 is not None else None
        wg = _native.edge_part_floats(1, P.shape[0], pc.n_items) // (32 * 34)
        part_w = torch.empty((wg, 32 * Wp.shape[1]), dtype=torch.float32, device=dev)
        _native.edge_epilogue_bwd(pc.items, pc.n_items, dPo, P, P0, ln_w, ln_b, ctx.eps, Wp, PROJ_SCALE, dSv,
                                  part_dsv, dP0, part_w)
        if not ctx.wp_by_cam:
            dWp = _native.param_colsum(part_w, ctx.defer).view(32, Wp.shape[1])
    if part_dsv is not None:
        bwd_combine(pc, part_dsv, 32, dSv)
    dSg_shared = dSg is not None
    dSg = _native.colsum(dSv, out=dSg)  # == d bias_proj: every edge belongs to one camera
    # point side: dSp = per-point sum of dP'/4 through the point permutation
    dSp = torch.empty((edges.n, 32), dtype=torch.float32, device=dev)
    part_dsp = torch.empty((max(pp.n_part_rows, 1), 32), dtype=torch.float32, device=dev)
    _native.segment_rowsum(pp.items, pp.n_items, pp.perm, dPo, PROJ_SCALE, dSp, part_dsp)
    bwd_combine(pp, part_dsp, 32, dSp)
    return (None, dP0, dPo, dSp, dSv, dSg.view(ctx.sg_shape), dWp,
            _bias_grad(dSv, dSg, getattr(ctx, "defer_b", False), shared=dSg_shared), None, None, None, None, None)


def _bias_grad(dSv, dSg, defer, shared=False):
    """lin_proj's bias gradient: the same column sum as dSg (every edge belongs to one camera), as
    its own tensor -- a deferred sum in the end-of-backward batch (no clone launch), or a clone of
    dSg.  shared: dSv / dSg are views of the boundary all-reduce's payload (_boundary_buffers),
    summed over the ranks IN PLACE before the pass ends, so the rank-local sum is taken now."""
    if defer and not shared:
        return _native.param_colsum(dSv, defer)[:]
    return dSg.clone()


class SeamFn(torch.autograd.Function):
    """Block b's EdgeEpilogueFn and block b+1's EdgeCamFn as ONE forward kernel
    (gasfm_edge_seam_fwd: P' is written once and never read back); the backward is the two
    Functions' own backwards in autograd's order (EdgeCamFn's, then EdgeEpilogueFn's on the
    resulting dP').

    Inputs: the 13 of EdgeEpilogueFn.forward, then the 20 of EdgeCamFn.forward (whose P is this
    Function's own output P').  Outputs: (P', XLp, camera aggregates, token).

    With EPI_FOLD and block b's lin_proj gradient taken by block b's own EdgeCamFn / SeamFn
    (wp_by_cam), the backward's edge_cam_pbwd also fills block b's dSv and dP0 from the dP' it
    produces, and edge_epilogue_bwd does not run."""

    @staticmethod
    def forward(ctx, P, P0, token, Sp, Sv, Sg, Wp, bp, lnw_b, lnb_b, eps_b, edges, wp_by_cam,
                ln_w, ln_b, Wpt, bpt, Wc, bc, Wp_n, eps, pos, XR, att, bias, plan, heads, slope, plan_partial, shard,
                P0_n=None, dwp_n=False):
        E, dev = P.shape[0], P.device
        HC = att.numel()
        if heads != 4 or HC != 32:
            raise ValueError("SeamFn: the fused kernels are for H = 4, C = 8")
        attf = att.reshape(-1).contiguous()
        XLp = torch.empty((E, 32), dtype=torch.float32, device=dev)
        Pn = torch.empty_like(P)
        Wp_c, Sp_c, Sv_r, Sg_f = Wp.contiguous(), Sp.contiguous(), _rows(Sv), Sg.reshape(-1).contiguous()
        bp_c = bp.contiguous()

        def launch(items, n_items, finalize, out, smax, ssum, part):
            _native.edge_seam_fwd(P, P0, edges.pt, lnw_b, lnb_b, eps_b, Wp_c, bp_c, Sp_c, Sv_r, Sg_f, PROJ_SCALE, Pn,
                                  ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, pos, XR, attf, bias if finalize else None,
                                  slope, items, n_items, finalize, out, smax, ssum, part)
        out, smax, ssum = _cam_attention_fwd(launch, bias, plan, heads, HC, plan_partial, shard, dev)
        # EdgeEpilogueFn's state
        ctx.e_eps, ctx.edges, ctx.sg_shape = eps_b, edges, Sg.shape
        ctx.e_wp_by_cam = bool(wp_by_cam)
        ctx.e_defer = _native.defer_token(Wp)
        ctx.e_defer_b = _native.defer_token(bp)
        # EdgeCamFn's state
        ctx.eps, ctx.heads, ctx.slope, ctx.plan = eps, heads, slope, plan
        ctx.att_shape = att.shape
        ctx.has_ln = ln_w is not None
        ctx.dwp = bool(dwp_n)
        ctx.sharded = shard is not None
        ctx.defer = _native.defer_token(ln_w, ln_b, Wpt, bpt, Wc, bc, att, bias, Wp_n if dwp_n else None)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(P, P0, Wp_c, lnw_b, lnb_b, Pn, ln_w, ln_b, Wpt, Wc, bc, Wp_n, XR, attf, bias, out, smax,
                              ssum, P0_n)
        ctx.n_epi = 5
        token_n = P.new_empty((1, 1)).expand(E, P.shape[1])
        return Pn, XLp, out, token_n

    @staticmethod
    def backward(ctx, gPn, dXLp, g_c, dtoken):
        saved = ctx.saved_tensors
        epi, cam = saved[:ctx.n_epi], saved[ctx.n_epi:]
        dRes = dtoken.contiguous() if (dtoken is not None and dtoken.stride(0) != 0) else None
        edges = ctx.edges
        dev = epi[0].device
        # sharded: block b's dSv / dSg and block b+1's camera target-row gradient, all partial per
        # rank, side by side in the one buffer the boundary all-reduce sums (AllReduceGradN: no cat)
        bnd = _boundary_buffers(edges.m, ctx.plan.num_targets, dev) if ctx.sharded else None
        folded = None
        if EPI_FOLD and ctx.e_wp_by_cam and gPn is None and ctx.plan is edges.plans["proj2view"]:
            # block b's dSv / dP0 from the dP' this launch produces (edge_cam_pbwd EPI)
            P_b, P0_b, Wp_b = epi[0], epi[1], epi[2]
            dSv = bnd[0] if bnd is not None else torch.empty((edges.m, 32), dtype=torch.float32, device=dev)
            part_dsv = torch.empty((max(ctx.plan.n_part_rows, 1), 32), dtype=torch.float32, device=dev)
            dP0 = torch.empty((P_b.shape[0], 2), dtype=torch.float32, device=dev) if P0_b is not None else None
            folded = (dSv, part_dsv, dP0)
        gc = _cam_backward(ctx, cam, dXLp, g_c, dRes, epi=None if folded is None else (Wp_b, PROJ_SCALE) + folded,
                           dXR=bnd[2] if bnd is not None else None)
        if not ctx.epi_done:
            folded = None
        elif ctx.epi_combined:
            folded = (folded[0], None, folded[2])
        dPn = gc[0] if gPn is None else gc[0] + gPn
        ectx = _EpiState(ctx.e_eps, edges, ctx.sg_shape, ctx.e_defer, ctx.e_wp_by_cam, ctx.e_defer_b)
        ge = _epilogue_backward(ectx, epi, dPn, folded,
                                dSg=bnd[1] if (bnd is not None and folded is not None) else None)
        return ge + gc[1:]


def _boundary_buffers(m, n_xr, dev):
    """(dSv [m, 32], dSg [32], dXR [n_xr, 32]) as consecutive views of ONE buffer: the payload of the
    point-sharded block boundary's all-reduce (distributed.AllReduceGradN sums it in place when its
    gradients arrive as these views, in this order)."""
    flat = torch.empty(m * 32 + 32 + n_xr * 32, dtype=torch.float32, device=dev)
    return flat[:m * 32].view(m, 32), flat[m * 32:m * 32 + 32], flat[m * 32 + 32:].view(n_xr, 32)


class _EpiState:
    def __init__(self, eps, edges, sg_shape, defer, wp_by_cam=False, defer_b=False):
        self.eps, self.edges, self.sg_shape, self.defer = eps, edges, sg_shape, defer
        self.wp_by_cam = wp_by_cam
        self.defer_b = defer_b


class PendingEpilogue:
    """Block b's EdgeEpilogueFn.apply arguments (block0: Block0EpilogueFn's), held so that block b+1
    can run it together with its own prologue (SeamFn / Seam0Fn); materialize() runs it alone (any
    other consumer of P')."""

    def __init__(self, args, block0=False):
        self.args = args
        self.block0 = block0
        self._P = None

    def seam_fn(self):
        return Seam0Fn if self.block0 else SeamFn

    def materialize(self):
        if self._P is None:
            self._P = (Block0EpilogueFn if self.block0 else EdgeEpilogueFn).apply(*self.args)
        return self._P


def materialize(P):
    return P.materialize() if isinstance(P, PendingEpilogue) else P


class Block0PrologueFn(torch.autograd.Function):
    """Block 0: XL0 = [Wl_pt; Wl_cam] relu(LN_a(P)) + b for 2-wide P (layers.py:232-234, 329, 426)."""

    @staticmethod
    def forward(ctx, P, ln_w, ln_b, W0, b0, eps, pos=None, perm=None):
        """pos (point plan's inverse permutation): write the point half of XL0 in point order.
        perm (the point plan's permutation, pos's inverse): the same XL0 written row by row."""
        E = P.shape[0]
        XL = torch.empty((E, 8), dtype=torch.float32, device=P.device)
        if pos is not None and perm is not None and E0_ROWS:
            _native.edge0_prologue_fwd_rows(P, ln_w, ln_b, eps, W0.contiguous(), b0.contiguous(), XL, perm)
        else:
            _native.edge0_prologue_fwd(P, ln_w, ln_b, eps, W0.contiguous(), b0.contiguous(), XL, pos)
        ctx.eps = eps
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(P, ln_w, ln_b, W0)
        return XL, P.new_empty((1, 1)).expand(E, 4)

    @staticmethod
    def backward(ctx, dXL, daux):
        P, ln_w, ln_b, W0 = ctx.saved_tensors
        E = P.shape[0]
        dXL = torch.zeros((E, 8), dtype=torch.float32, device=P.device) if dXL is None else dXL.contiguous()
        aux = daux.contiguous() if daux is not None and daux.stride(0) != 0 else None
        dP = torch.empty_like(P)
        rows = _native.edge0_part_rows(0, E)
        part = torch.empty((rows, 28), dtype=torch.float32, device=P.device)
        _native.edge0_prologue_bwd(dXL, P, aux, ln_w, ln_b, ctx.eps, W0.contiguous(), dP, part)
        tot = _native.colsum(part)
        return dP, tot[24:26], tot[26:28], tot[:16].view(8, 2), tot[16:24], None, None, None


class Block0EpilogueFn(torch.autograd.Function):
    """Block 0: P' = Wsk relu(LN_b(P)) + bsk + (Wp relu(LN_a(P)) + bp + Sp[pt] + Sv[cam] + Sg) / 4."""

    @staticmethod
    def forward(ctx, P, token, Sp, Sv, Sg, Wp, bp, lna_w, lna_b, lnb_w, lnb_b, Wsk, bsk, eps, edges):
        out = torch.empty((P.shape[0], Wp.shape[0]), dtype=torch.float32, device=P.device)
        _native.edge0_epilogue_fwd(P, edges.cam, edges.pt, lna_w, lna_b, lnb_w, lnb_b, eps, Wp.contiguous(),
                                   bp.contiguous(), Wsk.contiguous(), bsk.contiguous(), Sp.contiguous(),
                                   _rows(Sv), Sg.reshape(-1).contiguous(), PROJ_SCALE, out)
        ctx.eps, ctx.edges, ctx.sg_shape = eps, edges, Sg.shape
        ctx.defer_b = _native.defer_token(bp)
        ctx.save_for_backward(P, lna_w, lna_b, lnb_w, lnb_b, Wp, Wsk)
        return out

    @staticmethod
    def backward(ctx, dPo):
        return _epilogue0_backward(ctx, ctx.saved_tensors, dPo)


def _epilogue0_backward(ctx, saved, dPo, bnd=None):
    """Block0EpilogueFn's backward from its saved state (ctx attributes eps, edges, sg_shape,
    defer_b): its 15 input gradients.  bnd: the boundary all-reduce's (dSv, dSg, ...) views
    (_boundary_buffers) or None."""
    P, lna_w, lna_b, lnb_w, lnb_b, Wp, Wsk = saved
    edges = ctx.edges
    dPo = dPo.contiguous()
    dev = P.device
    E = P.shape[0]
    pc, pp = edges.plans["proj2view"], edges.plans["proj2scenepoint"]
    dSv = bnd[0] if bnd is not None else torch.empty((edges.m, 32), dtype=torch.float32, device=dev)
    part_dsv = torch.empty((max(pc.n_part_rows, 1), 32), dtype=torch.float32, device=dev)
    aux = torch.empty((E, 4), dtype=torch.float32, device=dev)
    rows = _native.edge0_part_rows(1, E, pc.n_items)
    part = torch.empty((rows, 164), dtype=torch.float32, device=dev)
    _native.edge0_epilogue_bwd(pc.items, pc.n_items, dPo, P, lna_w, lna_b, lnb_w, lnb_b, ctx.eps,
                               Wp.contiguous(), Wsk.contiguous(), PROJ_SCALE, dSv, part_dsv, aux, part)
    bwd_combine(pc, part_dsv, 32, dSv)
    tot = _native.colsum(part)
    dSg = _native.colsum(dSv, out=bnd[1] if bnd is not None else None)
    dSp = torch.empty((edges.n, 32), dtype=torch.float32, device=dev)
    part_dsp = torch.empty((max(pp.n_part_rows, 1), 32), dtype=torch.float32, device=dev)
    _native.segment_rowsum(pp.items, pp.n_items, pp.perm, dPo, PROJ_SCALE, dSp, part_dsp)
    bwd_combine(pp, part_dsp, 32, dSp)
    return (None, aux, dSp, dSv, dSg.view(ctx.sg_shape), tot[:64].view(32, 2),
            _bias_grad(dSv, dSg, getattr(ctx, "defer_b", False), shared=bnd is not None), None, None,
            tot[160:162], tot[162:164], tot[64:128].view(32, 2), tot[128:160], None, None)


class Seam0Fn(torch.autograd.Function):
    """Block 0's Block0EpilogueFn and block 1's EdgeCamFn as ONE forward kernel
    (gasfm_edge0_seam_fwd: P_1 is written once and never read back); the backward is the two
    Functions' own backwards in autograd's order.

    Inputs: the 15 of Block0EpilogueFn.forward, then the 19 of EdgeCamFn.forward after P (whose P
    is this Function's own output P_1).  Outputs: (P_1, XLp, camera aggregates, token)."""

    @staticmethod
    def forward(ctx, P, token, Sp, Sv, Sg, Wp, bp, lna_w, lna_b, lnb_w, lnb_b, Wsk, bsk, eps0, edges,
                ln_w, ln_b, Wpt, bpt, Wc, bc, Wp_n, eps, pos, XR, att, bias, plan, heads, slope, plan_partial, shard,
                P0_n=None, dwp_n=False):
        E, dev = P.shape[0], P.device
        HC = att.numel()
        if heads != 4 or HC != 32 or ln_w is None:
            raise ValueError("Seam0Fn: the fused kernels are for H = 4, C = 8 with the block's LayerNorm")
        attf = att.reshape(-1).contiguous()
        XLp = torch.empty((E, 32), dtype=torch.float32, device=dev)
        Pn = torch.empty((E, Wp.shape[0]), dtype=torch.float32, device=dev)
        Pc, Wp_c, Wsk_c = P.contiguous(), Wp.contiguous(), Wsk.contiguous()
        args0 = (Pc, edges.pt, lna_w, lna_b, lnb_w, lnb_b, eps0, Wp_c, bp.contiguous(), Wsk_c, bsk.contiguous(),
                 Sp.contiguous(), _rows(Sv), Sg.reshape(-1).contiguous(), PROJ_SCALE, Pn)

        def launch(items, n_items, finalize, out, smax, ssum, part):
            _native.edge0_seam_fwd(*args0, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, pos, XR, attf,
                                   bias if finalize else None, slope, items, n_items, finalize, out, smax, ssum, part)
        out, smax, ssum = _cam_attention_fwd(launch, bias, plan, heads, HC, plan_partial, shard, dev)
        # Block0EpilogueFn's state
        ctx.e_eps, ctx.edges, ctx.sg_shape = eps0, edges, Sg.shape
        ctx.e_defer_b = _native.defer_token(bp)
        # EdgeCamFn's state
        ctx.eps, ctx.heads, ctx.slope, ctx.plan = eps, heads, slope, plan
        ctx.att_shape = att.shape
        ctx.has_ln = True
        ctx.dwp = bool(dwp_n)
        ctx.sharded = shard is not None
        ctx.defer = _native.defer_token(ln_w, ln_b, Wpt, bpt, Wc, bc, att, bias, Wp_n if dwp_n else None)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(Pc, lna_w, lna_b, lnb_w, lnb_b, Wp_c, Wsk_c, Pn, ln_w, ln_b, Wpt, Wc, bc, Wp_n, XR,
                              attf, bias, out, smax, ssum, P0_n)
        token_n = P.new_empty((1, 1)).expand(E, Pn.shape[1])
        return Pn, XLp, out, token_n

    @staticmethod
    def backward(ctx, gPn, dXLp, g_c, dtoken):
        saved = ctx.saved_tensors
        epi, cam = saved[:7], saved[7:]
        dRes = dtoken.contiguous() if (dtoken is not None and dtoken.stride(0) != 0) else None
        edges = ctx.edges
        bnd = _boundary_buffers(edges.m, ctx.plan.num_targets, epi[0].device) if ctx.sharded else None
        gc = _cam_backward(ctx, cam, dXLp, g_c, dRes, dXR=bnd[2] if bnd is not None else None)
        dPn = gc[0] if gPn is None else gc[0] + gPn
        ectx = _EpiState(ctx.e_eps, edges, ctx.sg_shape, None, defer_b=ctx.e_defer_b)
        return _epilogue0_backward(ectx, epi, dPn, bnd) + gc[1:]
