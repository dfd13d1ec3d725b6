"""Scene-point side of a GASFM block as two fused autograd Functions (csrc/point_block.hip).

PointTailFn  -- the end of Proj2ScenePoint.forward (reference code/models/layers.py:438-454):
                x = prev + proj_proj2scenepoint(agg);  p = x + mlp(relu(norm_pre_mlp(x)))
PointHubFn   -- every consumer of the block output p, in one kernel forward and two backward:
                skip = p                                          next block's state skip (:442)
                SA   = lin_scenepoint(relu(scenepoint_norm_layer(p)))            (:928-935)
                XL   = graph_conv_scenepoint2global.lin_l(p)                     (:560-575, PyG)
                XR   = next.graph_conv.lin_r(next.norm_and_proj_scenepoint2proj(p))   (:429)

Why one Function for all consumers: autograd sums the gradients of a tensor with several
consumers using one full-size add per extra consumer ([n x 64], 51 MB at config 4, three per
block).  Routing every consumer through PointHubFn makes its backward the only producer of
dp: the C pass adds the next block's target-row gradient to the incoming skip gradient, the
A+B pass adds lin_l and lin_scenepoint terms in place, and no add kernel runs.
"""
import os

import torch

from . import _native

P_W = 64   # n_feat_scenepoint
A_W = 32   # n_feat_proj


def _f32(*shape, like):
    return torch.empty(shape, dtype=torch.float32, device=like.device)


class PointTailFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prev, agg, Wp, bp, ln_w, ln_b, Wm, bm, eps):
        agg = agg.contiguous()
        prev = prev.contiguous() if prev is not None else None
        Wp, Wm = Wp.contiguous(), Wm.contiguous()
        N = agg.shape[0]
        out = _f32(N, P_W, like=agg)
        _native.point_tail_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, bm, out)
        ctx.save_for_backward(prev, agg, Wp, bp, ln_w, ln_b, Wm)
        ctx.eps = eps
        ctx.defer = _native.defer_token(Wp, bp, ln_w, ln_b, Wm, bm)
        return out

    @staticmethod
    def backward(ctx, dout):
        return _tail_backward(ctx.saved_tensors, ctx.eps, ctx.defer, dout) + (None,)


def _tail_backward(saved, eps, defer, dout):
    """PointTailFn's backward: (d prev, d agg, dWp, dbp, dgamma, dbeta, dWm, dbm)."""
    prev, agg, Wp, bp, ln_w, ln_b, Wm = saved
    N = agg.shape[0]
    dout = dout.contiguous()
    rows, cols = _native.point_tail_part_shape(N, prev is not None)
    dx = _f32(N, P_W, like=agg)
    dagg = _f32(N, A_W, like=agg)
    if rows == 0:
        tot = torch.zeros(cols, dtype=torch.float32, device=agg.device)
    else:
        part = _f32(rows, cols, like=agg)
        _native.point_tail_bwd(dout, prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, dx, dagg, part)
        tot = _native.param_colsum(part, defer)
    o = 0
    dWm = tot[o:o + P_W * P_W].view(P_W, P_W)
    o += P_W * P_W
    dWp = tot[o:o + P_W * A_W].view(P_W, A_W)
    o += P_W * A_W
    dbm, dbp, dg, dbt = (tot[o + k * P_W:o + (k + 1) * P_W] for k in range(4))
    return (dx if prev is not None else None), dagg, dWp, dbp, dg, dbt, dWm, dbm


class PointHubFn(torch.autograd.Function):
    """p -> (skip, SA, XL, XR); see the module docstring for the four consumers."""

    @staticmethod
    def forward(ctx, p, gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD, eps):
        p = p.contiguous()
        WA, WB, WC, WD = (w.contiguous() for w in (WA, WB, WC, WD))
        N = p.shape[0]
        SA, XL, XR = _f32(N, A_W, like=p), _f32(N, P_W, like=p), _f32(N, A_W, like=p)
        _native.point_hub_fwd(p, eps, gA, bA, WA, SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR)
        ctx.save_for_backward(p, gA, bA, WA, WB, gC, bC, WC, bWC, WD)
        ctx.eps = eps
        ctx.defer = _native.defer_token(gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD)
        ctx.set_materialize_grads(False)
        return p.view_as(p), SA, XL, XR

    @staticmethod
    def backward(ctx, dskip, dSA, dXL, dXR):
        return _hub_backward(ctx.saved_tensors, ctx.eps, ctx.defer, dskip, dSA, dXL, dXR) + (None,)


def _hub_backward(saved, eps, defer, dskip, dSA, dXL, dXR):
    """PointHubFn's backward: (dp, dgA, dbA, dWA, dWB, dbB, dgC, dbC, dWC, dbWC, dWD, dbD); dp includes dskip."""
    p, gA, bA, WA, WB, gC, bC, WC, bWC, WD = saved
    N = p.shape[0]
    zeros = lambda w: torch.zeros((N, w), dtype=torch.float32, device=p.device)  # noqa: E731
    dSA = dSA.contiguous() if dSA is not None else zeros(A_W)
    dXL = dXL.contiguous() if dXL is not None else zeros(P_W)
    dXR = dXR.contiguous() if dXR is not None else zeros(A_W)
    dskip = dskip.contiguous() if dskip is not None else None
    rc, cc = _native.point_hub_part_shape(N, 1, dskip is not None)
    ra, ca = _native.point_hub_part_shape(N, 0, True)
    dp = _f32(N, P_W, like=p)
    if N == 0:
        tc = torch.zeros(cc, dtype=torch.float32, device=p.device)
        ta = torch.zeros(ca, dtype=torch.float32, device=p.device)
    else:
        part_c, part_a = _f32(rc, cc, like=p), _f32(ra, ca, like=p)
        _native.point_hub_bwd(p, eps, gA, bA, WA, WB, gC, bC, WC, bWC, WD, dSA, dXL, dXR, dskip, dp,
                              part_a, part_c)
        tc, ta = _native.param_colsum(part_c, defer), _native.param_colsum(part_a, defer)
    o = 0
    dWC = tc[o:o + A_W * P_W].view(A_W, P_W)
    o += A_W * P_W
    dWD = tc[o:o + A_W * A_W].view(A_W, A_W)
    o += A_W * A_W
    dbWC, dbD = tc[o:o + A_W], tc[o + A_W:o + 2 * A_W]
    o += 2 * A_W
    dgC, dbC = tc[o:o + P_W], tc[o + P_W:o + 2 * P_W]
    o = 0
    dWA = ta[o:o + A_W * P_W].view(A_W, P_W)
    o += A_W * P_W
    dWB = ta[o:o + P_W * P_W].view(P_W, P_W)
    o += P_W * P_W
    dbB, dgA, dbA = (ta[o + k * P_W:o + (k + 1) * P_W] for k in range(3))
    return dp, dgA, dbA, dWA, dWB, dbB, dgC, dbC, dWC, dbWC, dWD, dbD


class PointTailHubFn(torch.autograd.Function):
    """PointTailFn then PointHubFn on its output as ONE forward kernel (gasfm_point_tail_hub_fwd,
    round 6): p never re-read, one launch fewer per block.  Outputs (p, SA, XL, XR): p is the block's
    point features AND the next block's state skip (the hub's identity output), so its gradient --
    whatever consumes it -- enters the hub's backward as dRes.  The backward is the two Functions'
    own kernels in autograd's order (hub, then tail on the hub's dp)."""

    @staticmethod
    def forward(ctx, prev, agg, Wp, bp, ln_w, ln_b, Wm, bm, eps, gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD, eps_h):
        agg = agg.contiguous()
        prev = prev.contiguous() if prev is not None else None
        Wp, Wm, WA, WB, WC, WD = (w.contiguous() for w in (Wp, Wm, WA, WB, WC, WD))
        N = agg.shape[0]
        p = _f32(N, P_W, like=agg)
        SA, XL, XR = _f32(N, A_W, like=agg), _f32(N, P_W, like=agg), _f32(N, A_W, like=agg)
        _native.point_tail_hub_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, bm, p, eps_h, gA, bA, WA, SA, WB, bB, XL,
                                   gC, bC, WC, bWC, WD, bD, XR)
        ctx.save_for_backward(prev, agg, Wp, bp, ln_w, ln_b, Wm, p, gA, bA, WA, WB, gC, bC, WC, bWC, WD)
        ctx.eps, ctx.eps_h = eps, eps_h
        ctx.defer_t = _native.defer_token(Wp, bp, ln_w, ln_b, Wm, bm)
        ctx.defer_h = _native.defer_token(gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD)
        ctx.set_materialize_grads(False)
        return p, SA, XL, XR

    @staticmethod
    def backward(ctx, dp, dSA, dXL, dXR):
        saved = ctx.saved_tensors
        gh = _hub_backward(saved[7:], ctx.eps_h, ctx.defer_h, dp, dSA, dXL, dXR)
        gt = _tail_backward(saved[:7], ctx.eps, ctx.defer_t, gh[0])
        return gt[:8] + (None,) + gh[1:] + (None,)


def _is_ln(m, w):
    return isinstance(m, torch.nn.LayerNorm) and tuple(m.normalized_shape) == (w,) and m.weight is not None \
        and m.bias is not None


def _is_lin(m, i, o, bias):
    return isinstance(m, torch.nn.Linear) and m.in_features == i and m.out_features == o \
        and ((m.bias is not None) == bias)


def _rows_ok(t, w):
    return t is not None and t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape[1] == w


def tail_fusable(agg_mod, x, prev):
    """Proj2ScenePoint with 32-wide aggregation, 64-wide points, norm_pre_mlp and a one-Linear mlp."""
    if not (_rows_ok(x, A_W) and (prev is None or _rows_ok(prev, P_W))):
        return False
    proj = getattr(agg_mod, agg_mod._proj_key, None) if agg_mod.n_feat_agg != agg_mod.n_feat_out else None
    return (proj is not None and _is_lin(proj, A_W, P_W, True) and agg_mod.use_norm_pre_mlp
            and _is_ln(agg_mod.norm_pre_mlp, P_W) and len(agg_mod.mlp) == 1 and _is_lin(agg_mod.mlp[0], P_W, P_W, True))


def tail(agg_mod, x, prev):
    proj = getattr(agg_mod, agg_mod._proj_key)
    ln, lin = agg_mod.norm_pre_mlp, agg_mod.mlp[0]
    return PointTailFn.apply(prev, x, proj.weight, proj.bias, ln.weight, ln.bias, lin.weight, lin.bias, ln.eps)


def hub_params(pfu, s2g_conv, nxt):
    """(gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD, eps) or None when the shapes do not match.

    pfu: this block's projection-feature update (scenepoint_norm_layer, lin_scenepoint);
    s2g_conv: this block's graph_conv_scenepoint2global; nxt: the next Proj2ScenePoint."""
    if pfu is None or s2g_conv is None or nxt is None or not pfu.normalize_global_features:
        return None
    lnA, linA = pfu.scenepoint_norm_layer, pfu.lin_scenepoint
    linB = s2g_conv.lin_l
    seq = getattr(nxt, nxt._state_key, None) if nxt.stateful else None
    if seq is None or len(seq) != 3:
        return None
    lnC, linC, linD = seq[0], seq[2], nxt.graph_conv.lin_r
    if not (_is_ln(lnA, P_W) and _is_lin(linA, P_W, A_W, False) and _is_lin(linB, P_W, P_W, True)
            and _is_ln(lnC, P_W) and _is_lin(linC, P_W, A_W, True) and _is_lin(linD, A_W, A_W, True)
            and lnA.eps == lnC.eps):
        return None
    return (lnA.weight, lnA.bias, linA.weight, linB.weight, linB.bias, lnC.weight, lnC.bias, linC.weight,
            linC.bias, linD.weight, linD.bias, lnA.eps)


def hub(p, params):
    return PointHubFn.apply(p, *params)


# round 6: the tail and the hub as one forward launch (PointTailHubFn); GASFM_TAIL_HUB=0 runs the two
# Functions (A/B knob)
FUSED_TAIL_HUB = os.environ.get("GASFM_TAIL_HUB", "1") != "0"


def tail_hub(agg_mod, x, prev, params):
    """(p, skip, SA, XL, XR) of tail() then hub() -- one forward kernel; skip IS p (see PointTailHubFn)."""
    proj = getattr(agg_mod, agg_mod._proj_key)
    ln, lin = agg_mod.norm_pre_mlp, agg_mod.mlp[0]
    gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD, eps_h = params
    p, SA, XL, XR = PointTailHubFn.apply(prev, x, proj.weight, proj.bias, ln.weight, ln.bias, lin.weight, lin.bias,
                                         ln.eps, gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD, eps_h)
    return p, p, SA, XL, XR


class PointHeadFn(torch.autograd.Function):
    """pts3D = [scenepoint_head(relu(p))^T ; 1] (reference code/models/graph_attn_sfm.py:170-174)
    in one forward kernel and two backward kernels (csrc/point_head.hip); the scene-point head
    is Linear(64,64) ReLU Linear(64,64) ReLU Linear(64,3) (layers.py:10-44, norm=False)."""

    @staticmethod
    def forward(ctx, p, W1, b1, W2, b2, W3, b3):
        p = p.contiguous()
        N = p.shape[0]
        out = _f32(4, N, like=p)
        _native.point_head_fwd(p, W1, b1, W2, b2, W3, b3, out)
        ctx.save_for_backward(p, W1, b1, W2, b2, W3)
        ctx.defer = _native.defer_token(W1, b1, W2, b2, W3, b3)
        return out

    @staticmethod
    def backward(ctx, dout):
        p, W1, b1, W2, b2, W3 = ctx.saved_tensors
        N = p.shape[0]
        ra, ca = _native.point_head_part_shape(N, 0)
        rb, cb = _native.point_head_part_shape(N, 1)
        dp = _f32(N, P_W, like=p)
        if N == 0:
            ta = torch.zeros(ca, dtype=torch.float32, device=p.device)
            tb = torch.zeros(cb, dtype=torch.float32, device=p.device)
        else:
            part_a, part_b = _f32(ra, ca, like=p), _f32(rb, cb, like=p)
            _native.point_head_bwd(p, W1, b1, W2, b2, W3, dout.contiguous(), dp, part_a, part_b)
            ta, tb = _native.param_colsum(part_a, ctx.defer), _native.param_colsum(part_b, ctx.defer)
        dW1, db1 = ta[:P_W * P_W].view(P_W, P_W), ta[P_W * P_W:]
        o = P_W * P_W
        dW2, dW3 = tb[:o].view(P_W, P_W), tb[o:o + 3 * P_W].view(3, P_W)
        o += 3 * P_W
        db2, db3 = tb[o:o + P_W], tb[o + P_W:o + P_W + 3]
        return dp, dW1, db1, dW2, db2, dW3, db3


def head_fusable(seq, p):
    """The configuration's scene-point head: two 64-wide hidden layers, 3 outputs, no norms."""
    mods = list(seq)
    return (_rows_ok(p, P_W) and len(mods) == 5 and _is_lin(mods[0], P_W, P_W, True)
            and isinstance(mods[1], torch.nn.ReLU) and _is_lin(mods[2], P_W, P_W, True)
            and isinstance(mods[3], torch.nn.ReLU) and _is_lin(mods[4], P_W, 3, True)
            and all(m.weight.dtype == torch.float32 and m.weight.is_contiguous() and m.bias.is_contiguous()
                    for m in (mods[0], mods[2], mods[4])))


def head(seq, p):
    l1, l2, l3 = seq[0], seq[2], seq[4]
    return PointHeadFn.apply(p, l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias)
