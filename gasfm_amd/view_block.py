"""Camera (view) side of a GASFM block as two fused autograd Functions (csrc/view_block.hip).

ViewTailFn -- the end of Proj2View.forward (reference code/models/layers.py:345-360):
              x = prev + proj_proj2view(agg);  view = x + mlp(relu(norm_pre_mlp(x)))
              one kernel for x / x + b_m / relu(LN(x)), one hipBLASLt GEMM (addmm) for mlp.
ViewHubFn  -- every consumer of the block's view features, as PointHubFn does for points
              (point_block.py): the identity skip to the next block, lin_view(relu(view_norm_layer)),
              the next block's lin_r(norm_and_proj_view2proj(view)) (one kernel) and
              graph_conv_view2global.lin_l (addmm).  Its backward is the only producer of d view:
              addmm(d skip, dXL, W_l) then one kernel adding both LayerNorm branches in place.

The two D x D GEMMs of the camera side (m = 1000 rows, D = 1024) run on hipBLASLt through torch
in fp32, or -- BASELINE config 5's "bf16 projections on MFMA", ``bf16=True`` -- on the hand-written
bf16 MFMA kernel (csrc/gemm_bf16.hip: operands rounded to bf16, fp32 accumulation, bias / skip
fused), forward and both backward products.  Everything around them -- LayerNorms, ReLUs, the
32-wide projections, residual adds, bias / LayerNorm-affine gradient reductions -- runs in the
four kernels.
"""
import os

import torch

from . import _native

A_W = 32
WIDTHS = tuple(range(64, 1025, 64))  # D: a multiple of 64 (one wave per 64 columns), <= 1024
TR = 16


def _f32(*shape, like):
    return torch.empty(shape, dtype=torch.float32, device=like.device)


# fp32 camera-side GEMMs: "torch" = hipBLASLt (default), "hip" = csrc/gemm_f32.hip.  Measured
# (tools/gemm_bench.py, MI355X): at m = 1000 hipBLASLt 25-28 us vs 35-43 us for the HIP kernel;
# at m = 125 the HIP kernel 12-16 us vs 19 us standalone, but the whole emulated rank-of-8 step
# 10.33 ms vs 9.97 ms with hipBLASLt, so hipBLASLt stays the default.
FP32_GEMM = os.environ.get("GASFM_VIEW_GEMM", "torch")
# fp32 products with at most this many camera rows (a camera-sharded rank's 125, a training
# batch's ~60) go to csrc/gemm_smallm.hip (1,024 waves of 16 x 32 tiles x K-quarters) instead of
# hipBLASLt, whose 125 x 1024 x 1024 tiles take ~11.5 us; 0 disables
SMALLM_ROWS = int(os.environ.get("GASFM_SMALLM_ROWS", "256"))
# fp32 camera sides of at most 256 rows (view_chain_ok) run as csrc/view_chain.hip: the D x D GEMMs
# with the view kernels as their prologues / epilogues, 2 launches forward and 4 backward per block
# (round 3: 7 and 10); GASFM_VIEW_CHAIN=0 keeps the separate view kernels + GEMMs
VIEW_CHAIN = os.environ.get("GASFM_VIEW_CHAIN", "1") != "0"
# GASFM_WGRAD_GEMM=hip: the camera-side weight gradients dW = dy^T x above SMALLM_ROWS rows on
# csrc/gemm_f32.hip's direct-to-LDS kernel (round 6: 26.9 vs 27.9 us standalone at m = 1000, but the
# config-4 step 28.22-28.29 vs 28.18-28.20 ms with hipBLASLt on the same box, profiles/r6_gemm_f32.txt)
WGRAD_HIP = os.environ.get("GASFM_WGRAD_GEMM", "torch") == "hip"


def _chain_ok(m, D, bf16):
    """The fused small-m view chain (vc_* kernels, fp32 products) runs whenever it fits, in the bf16
    projection mode too: at its row counts (a camera-sharded rank's ~125 rows, a training batch's
    ~60) the separate bf16 GEMM launches are latency-bound and slower (rank-0-of-8: 8.67 vs 7.66 ms,
    round 5), so bf16 applies to the large-m GEMM path only."""
    return VIEW_CHAIN and FP32_GEMM == "torch" and m > 0 and _native.view_chain_ok(m, D)


def _mm(a, b, cin=None, bias=None, bf16=False, out=None):
    """a @ b (+ cin) (+ bias): the bf16 MFMA kernel, the fp32 MFMA kernel or fp32 hipBLASLt;
    out may be cin (accumulate in place)."""
    if bf16:
        return _native.gemm_bf16(a, b, cin=cin, bias=bias, out=out)
    if FP32_GEMM == "hip":
        return _native.gemm_f32(a, b, cin=cin, bias=bias, out=out)
    # the row count is a's rows (x W^T, dy W) or the shared K (dy^T x)
    rows = a.shape[0] if a.stride(1) == 1 else a.shape[1]
    if rows <= SMALLM_ROWS:
        y = _native.gemm_f32_smallm(a, b, cin=cin, bias=bias, out=out)
        if y is not None:
            return y
    elif WGRAD_HIP and a.stride(0) == 1 and cin is None and bias is None:
        # dW = dy^T x over > SMALLM_ROWS camera rows on csrc/gemm_f32.hip (opt-in, above)
        return _native.gemm_f32(a, b, out=out)
    if cin is not None:
        if out is cin and bias is None:
            return cin.addmm_(a, b)
        return torch.addmm(cin if bias is None else cin + bias, a, b, out=out)
    return torch.addmm(bias, a, b, out=out) if bias is not None else torch.mm(a, b, out=out)


class ViewTailFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prev, agg, Wp, bp, ln_w, ln_b, Wm, bm, eps, bf16=False, exch=None):
        """exch (distributed.BlockExchange): the backward writes d agg straight into the block's
        backward send block (the camera-sharded own-row gather)."""
        agg = agg.contiguous()
        prev = prev.contiguous() if prev is not None else None
        Wp, Wm = Wp.contiguous(), Wm.contiguous()
        m, D = agg.shape[0], Wp.shape[0]
        x, h = _f32(m, D, like=agg), _f32(m, D, like=agg)
        rs = _f32(m, 2, like=agg)
        ctx.chain = _chain_ok(m, D, bf16)
        if ctx.chain:
            view = _f32(m, D, like=agg)
            _native.view_chain_tail_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, bm, view, x, h, rs)
        else:
            xb = _f32(m, D, like=agg)
            _native.view_tail_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, bm, x, xb, h, rs,
                                  _native.view_scratch(m, D, agg.device))
            # xb + h Wm^T accumulated in place (torch's addmm with a separate input first copies it)
            view = _mm(h, Wm.t(), cin=xb, bf16=bf16, out=xb)
        ctx.save_for_backward(agg, x, rs, h, Wp, ln_w, ln_b, Wm)
        ctx.eps, ctx.has_prev, ctx.bf16 = eps, prev is not None, bf16
        ctx.exch = exch
        ctx.defer = _native.defer_token(Wp, bp, ln_w, ln_b, bm)
        return view

    @staticmethod
    def backward(ctx, dview):
        agg, x, rs, h, Wp, ln_w, ln_b, Wm = ctx.saved_tensors
        m, D = x.shape
        dview = dview.contiguous()
        ex, ctx.exch = ctx.exch, None
        if ctx.chain:
            dh, dx = _f32(m, D, like=x), _f32(m, D, like=x)
            dagg = ex.dagg_out() if (ex is not None and ex.own == m) else _f32(m, A_W, like=x)
            dWm = torch.empty_like(Wm)
            part = _f32((m + TR - 1) // TR, _native.view_tail_part_cols(D), like=x)
            _native.view_chain_tail_bwd(dview, x, h, rs, agg, Wp, ln_w, ln_b, Wm, dh, dWm, dx, dagg, part)
            tot = _native.param_colsum(part, ctx.defer)
            dWp = tot[:D * A_W].view(D, A_W)
            dbp, dg, dbt, dbm = (tot[D * A_W + k * D:D * A_W + (k + 1) * D] for k in range(4))
            return (dx if ctx.has_prev else None), dagg, dWp, dbp, dg, dbt, dWm, dbm, None, None, None
        dh = _mm(dview, Wm, bf16=ctx.bf16)
        dWm = _mm(dview.t(), h, bf16=ctx.bf16)
        dx = _f32(m, D, like=x)
        dagg = ex.dagg_out() if (ex is not None and ex.own == m) else _f32(m, A_W, like=x)
        cols = _native.view_tail_part_cols(D)
        if m == 0:
            tot = torch.zeros(cols, dtype=torch.float32, device=x.device)
        else:
            part = _f32((m + TR - 1) // TR, cols, like=x)
            _native.view_tail_bwd(dview, dh, x, rs, agg, Wp, ln_w, ln_b, dx, dagg, part,
                                  _native.view_scratch(m, D, x.device))
            tot = _native.param_colsum(part, ctx.defer)
        dWp = tot[:D * A_W].view(D, A_W)
        dbp, dg, dbt, dbm = (tot[D * A_W + k * D:D * A_W + (k + 1) * D] for k in range(4))
        return (dx if ctx.has_prev else None), dagg, dWp, dbp, dg, dbt, dWm, dbm, None, None, None


class ViewHubFn(torch.autograd.Function):
    """v -> (skip, SV, XL, XR)."""

    @staticmethod
    def forward(ctx, v, gC, bC, Wv, Wl, bl, gA, bA, Wa, ba, Wr, br, eps, bf16=False, packed=False, out=None):
        """packed: SV and XR are the two column halves of one [m, 64] block (the camera-sharded
        path all-gathers that block as it is); out: that block's [m, 64] destination (the block
        exchange's send block, distributed.BlockExchange)."""
        v = v.contiguous()
        Wv, Wl, Wa, Wr = (w.contiguous() for w in (Wv, Wl, Wa, Wr))
        m = v.shape[0]
        t = _f32(m, A_W, like=v)
        if packed:
            blk = out if out is not None else _f32(m, 2 * A_W, like=v)
            SV, XR = blk[:, :A_W], blk[:, A_W:]
        else:
            SV, XR = _f32(m, A_W, like=v), _f32(m, A_W, like=v)
        rs = _f32(m, 2, like=v)
        ctx.chain = _chain_ok(m, v.shape[1], bf16)
        if ctx.chain:
            XL = _f32(m, Wl.shape[0], like=v)
            _native.view_chain_hub_fwd(v, eps, Wl, bl, gC, bC, Wv, gA, bA, Wa, ba, Wr, br, XL, SV, t, XR, rs)
        else:
            _native.view_hub_fwd(v, eps, gC, bC, Wv, gA, bA, Wa, ba, Wr, br, SV, t, XR, rs,
                                 _native.view_scratch(m, v.shape[1], v.device))
            XL = _mm(v, Wl.t(), bias=bl, bf16=bf16)
        ctx.save_for_backward(v, rs, t, gC, bC, Wv, Wl, gA, bA, Wa, Wr)
        ctx.eps, ctx.bf16 = eps, bf16
        ctx.defer = _native.defer_token(gC, bC, Wv, gA, bA, Wa, ba, Wr, br, bl)
        ctx.set_materialize_grads(False)
        return v.view_as(v), SV, XL, XR

    @staticmethod
    def backward(ctx, dskip, dSV, dXL, dXR):
        v, rs, t, gC, bC, Wv, Wl, gA, bA, Wa, Wr = ctx.saved_tensors
        m, D = v.shape
        zeros = lambda w: torch.zeros((m, w), dtype=torch.float32, device=v.device)  # noqa: E731
        dSV = dSV.contiguous() if dSV is not None else zeros(A_W)
        dXR = dXR.contiguous() if dXR is not None else zeros(A_W)
        dXL = dXL.contiguous() if dXL is not None else zeros(D)
        dres = None
        if ctx.chain:
            dacc, dWl = _f32(m, D, like=v), torch.empty_like(Wl)
            part = _f32((m + TR - 1) // TR, _native.view_hub_part_cols(D), like=v)
            _native.view_chain_hub_bwd(v, rs, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dSV, dXR, dXL,
                                       dskip.contiguous() if dskip is not None else None, dacc, dWl, part)
            tot = _native.param_colsum(part, ctx.defer)
        elif ctx.bf16 or FP32_GEMM == "hip":  # the MFMA kernels add d skip in their epilogue
            dacc = _mm(dXL, Wl, cin=dskip.contiguous() if dskip is not None else None, bf16=ctx.bf16)
        else:  # hipBLASLt: d skip is added by the hub kernel's second pass (no addmm input copy)
            dacc = _mm(dXL, Wl)
            dres = dskip.contiguous() if dskip is not None else None
        if not ctx.chain:
            dWl = _mm(dXL.t(), v, bf16=ctx.bf16)
            cols = _native.view_hub_part_cols(D)
            if m == 0:
                tot = torch.zeros(cols, dtype=torch.float32, device=v.device)
            else:
                part = _f32((m + TR - 1) // TR, cols, like=v)
                _native.view_hub_bwd(v, rs, gC, bC, Wv, gA, bA, Wa, t, Wr, dSV, dXR, dXL, dacc, part,
                                     _native.view_scratch(m, D, v.device), dres=dres)
                tot = _native.param_colsum(part, ctx.defer)
        o = 0
        dWv = tot[o:o + A_W * D].view(A_W, D)
        o += A_W * D
        dWa = tot[o:o + A_W * D].view(A_W, D)
        o += A_W * D
        dgC, dbC, dgA, dbA, dbl = (tot[o + k * D:o + (k + 1) * D] for k in range(5))
        o += 5 * D
        dWr = tot[o:o + A_W * A_W].view(A_W, A_W)
        o += A_W * A_W
        dba, dbr = tot[o:o + A_W], tot[o + A_W:o + 2 * A_W]
        return dacc, dgC, dbC, dWv, dWl, dbl, dgA, dbA, dWa, dba, dWr, dbr, None, None, None, None


def _is_ln(mod, w):
    return isinstance(mod, torch.nn.LayerNorm) and tuple(mod.normalized_shape) == (w,) and mod.weight is not None \
        and mod.bias is not None


def _is_lin(mod, i, o, bias):
    return isinstance(mod, torch.nn.Linear) and mod.in_features == i and mod.out_features == o \
        and ((mod.bias is not None) == bias)


def _rows_ok(t, w):
    return t is not None and t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.shape[1] == w


def tail_fusable(agg_mod, x, prev):
    """Proj2View with 32-wide aggregation, D-wide views (D in WIDTHS), norm_pre_mlp and a
    one-Linear mlp."""
    D = agg_mod.n_feat_out
    if D not in WIDTHS or not (_rows_ok(x, A_W) and (prev is None or _rows_ok(prev, D))):
        return False
    proj = getattr(agg_mod, agg_mod._proj_key, None) if agg_mod.n_feat_agg != D else None
    return (proj is not None and _is_lin(proj, A_W, D, True) and agg_mod.use_norm_pre_mlp
            and _is_ln(agg_mod.norm_pre_mlp, D) and len(agg_mod.mlp) == 1 and _is_lin(agg_mod.mlp[0], D, D, True))


def tail(agg_mod, x, prev, exch=None):
    proj = getattr(agg_mod, agg_mod._proj_key)
    ln, lin = agg_mod.norm_pre_mlp, agg_mod.mlp[0]
    return ViewTailFn.apply(prev, x, proj.weight, proj.bias, ln.weight, ln.bias, lin.weight, lin.bias, ln.eps,
                            getattr(agg_mod, "_proj_bf16", False), exch)


def hub_params(pfu, v2g_conv, nxt):
    """(gC, bC, Wv, Wl, bl, gA, bA, Wa, ba, Wr, br, eps) or None when the shapes do not match.

    pfu: this block's projection-feature update (view_norm_layer, lin_view); v2g_conv: this
    block's graph_conv_view2global; nxt: the next Proj2View (norm_and_proj_view2proj, lin_r)."""
    if pfu is None or v2g_conv is None or nxt is None or not pfu.normalize_global_features or not nxt.stateful:
        return None
    lnC, linV = pfu.view_norm_layer, pfu.lin_view
    D = linV.in_features
    seq = getattr(nxt, nxt._state_key, None)
    if D not in WIDTHS or seq is None or len(seq) != 3:
        return None
    lnA, linA, linR, linL = seq[0], seq[2], nxt.graph_conv.lin_r, v2g_conv.lin_l
    if not (_is_ln(lnC, D) and _is_lin(linV, D, A_W, False) and _is_lin(linL, D, D, True) and _is_ln(lnA, D)
            and _is_lin(linA, D, A_W, True) and _is_lin(linR, A_W, A_W, True) and lnA.eps == lnC.eps):
        return None
    return (lnC.weight, lnC.bias, linV.weight, linL.weight, linL.bias, lnA.weight, lnA.bias, linA.weight, linA.bias,
            linR.weight, linR.bias, lnC.eps)


def hub(v, params, bf16=False, packed=False, out=None):
    return ViewHubFn.apply(v, *params, bf16, packed, out)
