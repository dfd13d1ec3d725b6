"""Dense per-node layers (point rows: n ~ 200k) with a split-K weight gradient.

torch's Linear backward computes dW = dY^T X as ONE GEMM with K = rows; for the
GASFM point layers (M, N <= 64, K = 200k) hipBLASLt then runs one or two
workgroups (measured 0.45-0.53 ms per call on MI355X, ~40 ms per training
step), and for the camera layers (32x1024 / 1024x32 weights, K = 1000 cameras)
24-48 workgroups at 39-56 us per call.  ``linear`` keeps torch's forward /
input-gradient GEMMs (MFMA through hipBLASLt, good shapes) and computes the weight
gradient as a batched GEMM over row chunks followed by a sum (split-K), which fills
the chip.
The single global row goes through csrc/global_vec.hip (GlobalLinearFn).
"""
import weakref

import torch
import torch.nn.functional as F
from torch.nn import LayerNorm, Linear, ReLU, Sequential

SPLITK_MIN_ROWS = 256      # camera rows (m ~ 1000) and point rows (n ~ 200k)
_MIN_CHUNK = 128           # rows per split-K slice at least ...
_MAX_SLICES = 256          # ... and at most this many slices: a 32x64 weight gradient is only a
                           # few output tiles, so the slice count sets the workgroup count (12
                           # slices of 2k rows ran 24 workgroups at 55 us per call)


def _colsum(a):
    """Column sums of a 2-D CUDA tensor: the one-launch gasfm_colsum for short, wide inputs
    (split-K slices, camera rows); gasfm_colsum_tall for tall, narrow ones (E edge or 200k
    point rows), where colsum's <= 64 row blocks per column chunk would leave the chip idle.
    Not torch's sum: its global reduction replayed from a captured hipGraph gave wrong sums
    (DESIGN.md §5)."""
    from . import _native
    a = a.contiguous()
    if a.shape[0] > 4096 and _native.colsum_tall_ok(a):
        return _native.colsum_tall(a)
    return _native.colsum(a)


def bias_colsum(dy, defer):
    """A bias gradient (column sum of dy [rows, n]) as a VIEW of its sum tensor: deferred into the
    end-of-backward batched parameter sums (_native.param_colsum) for camera-sized inputs, at once
    through _colsum's tall kernel for edge / point-sized ones.  AccumulateGrad adopts a view; it
    would copy a pending (not yet filled) sum tensor itself (edge_block.replicated_dbias)."""
    from . import _native
    return (_native.param_colsum(dy, defer) if dy.shape[0] <= 4096 else _colsum(dy))[:]


def splitk_wgrad(dy, x):
    R, M = dy.shape
    N = x.shape[1]
    if R <= 4096 or (R < 16384 and M * N > 262144):
        # camera rows (m <= 4096): one GEMM beats the slices + column sum (7.5 vs 16.7 us at 1000 x
        # 1024 x 4, tools/wgrad_bench.py); camera 1024x1024 weights: already 256 output tiles
        return dy.T @ x
    B = max(1, min(_MAX_SLICES, R // _MIN_CHUNK))
    if B == 1:
        return dy.T @ x
    R0 = (R // B) * B
    dW = _colsum(torch.bmm(dy[:R0].reshape(B, R0 // B, M).transpose(1, 2), x[:R0].reshape(B, R0 // B, N))
                 .reshape(B, M * N)).view(M, N)
    if R0 < R:
        dW = dW + dy[R0:].T @ x[R0:]
    return dW


class RowLinearFn(torch.autograd.Function):
    """y = x W^T + b on device rows: the weight gradient split-K over tall inputs, the bias
    gradient a column sum deferred into the end-of-backward batch (_native.param_colsum; aten's
    addmm backward runs a reduce plus a memset launch per Linear)."""

    @staticmethod
    def forward(ctx, x, W, b):
        from . import _native
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        ctx.defer = _native.defer_token(b) if b is not None else False
        return F.linear(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy @ W if ctx.needs_input_grad[0] else None
        dW = splitk_wgrad(dy, x.contiguous()) if ctx.needs_input_grad[1] else None
        db = bias_colsum(dy, ctx.defer) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dW, db


class GlobalLinearFn(torch.autograd.Function):
    """ONE row: y = W h + b (+ res, or + x when resid_x), h = relu(LN(x)) when ln_w is given.

    The global node's GEMV chains (csrc/global_vec.hip): one kernel forward, a slab pass plus
    a one-workgroup finish backward, instead of LayerNorm/clamp/M=1 GEMM/add kernels."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, W, b, res, eps, resid_x):
        from . import _native
        x1 = x.reshape(-1).contiguous()
        W = W.contiguous()
        y = torch.empty((1, W.shape[0]), dtype=torch.float32, device=x.device)
        r = x1 if resid_x else (res.reshape(-1).contiguous() if res is not None else None)
        _native.gvec_fwd(x1, ln_w, ln_b, eps, W, b, r, y)
        ctx.save_for_backward(x1, ln_w, ln_b, W)
        ctx.eps, ctx.resid_x = eps, resid_x
        ctx.has_b, ctx.has_res, ctx.x_shape = b is not None, res is not None, x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _native
        x1, ln_w, ln_b, W = ctx.saved_tensors
        N, K = W.shape
        dy1 = dy.reshape(-1).contiguous()
        dev = x1.device
        f = dict(dtype=torch.float32, device=dev)
        dx = torch.empty(K, **f)
        dW = torch.empty_like(W)
        db = torch.empty(N, **f) if ctx.has_b else None
        dg = torch.empty(K, **f) if ln_w is not None else None
        dbt = torch.empty(K, **f) if ln_w is not None else None
        part = torch.empty((_native.gvec_bwd_chunks(N), K), **f)
        _native.gvec_bwd(dy1, x1, ln_w, ln_b, ctx.eps, W, ctx.resid_x, dx, dW, db, dg, dbt, part)
        dres = dy if ctx.has_res else None
        return dx.view(ctx.x_shape), dg, dbt, dW, db, dres, None, None


GVEC_MAX_K = 4096


class GlobalHubFn(torch.autograd.Function):
    """Every consumer of a block's global row g [1, G] in two launches each way.

    (skip, SG, XRv, XRp) with
      SG  = lin_global(relu(global_norm_layer(g)))              this block's projection update
      XRv = lin_r_v(norm_and_proj_global2view(g))               next block's view2global target row
      XRp = lin_r_p(norm_and_proj_global2scenepoint(g))         next block's scenepoint2global target row
      skip = g                                                  next block's proj_view_and_scenepoint2global residual
    (layers.py:497-520, 527-528, 590-592, 928-935).  Forward: the three LayerNorm -> Linear rows in one
    batched gvec launch, the two lin_r rows in a second.  Backward: the lin_r rows (batched), then the
    three LayerNorm rows with their dg contributions and the skip gradient summed in one finish pass --
    no autograd accumulation over g's four consumers.
    """

    @staticmethod
    def forward(ctx, g, gA, bA, WA, gB, bB, WB, bWB, gC, bC, WC, bWC, WD, bD, WE, bE, eps):
        from . import _native
        g1 = g.reshape(-1).contiguous()
        W = [w.contiguous() for w in (WA, WB, WC, WD, WE)]
        f = dict(dtype=torch.float32, device=g.device)
        sg, xv, xp = torch.empty(W[0].shape[0], **f), torch.empty(W[1].shape[0], **f), torch.empty(W[2].shape[0], **f)
        XRv, XRp = torch.empty(W[3].shape[0], **f), torch.empty(W[4].shape[0], **f)
        _native.gvec_multi_fwd([(g1, gA, bA, W[0], None, None, sg), (g1, gB, bB, W[1], bWB, None, xv),
                                (g1, gC, bC, W[2], bWC, None, xp)], eps)
        _native.gvec_multi_fwd([(xv, None, None, W[3], bD, None, XRv), (xp, None, None, W[4], bE, None, XRp)], 0.0)
        ctx.save_for_backward(g1, xv, xp, gA, bA, gB, bB, gC, bC, *W)
        ctx.eps, ctx.g_shape = eps, g.shape
        ctx.set_materialize_grads(False)
        return g.view_as(g), sg.view(1, -1), XRv.view(1, -1), XRp.view(1, -1)

    @staticmethod
    def backward(ctx, dskip, dsg, dXRv, dXRp):
        from . import _native
        g1, xv, xp, gA, bA, gB, bB, gC, bC, WA, WB, WC, WD, WE = ctx.saved_tensors
        f = dict(dtype=torch.float32, device=g1.device)
        row = lambda t, n: t.reshape(-1).contiguous() if t is not None else torch.zeros(n, **f)  # noqa: E731
        dsg, dXRv, dXRp = row(dsg, WA.shape[0]), row(dXRv, WD.shape[0]), row(dXRp, WE.shape[0])
        dres = dskip.reshape(-1).contiguous() if dskip is not None else None
        part = lambda W: torch.empty((_native.gvec_bwd_chunks(W.shape[0]), W.shape[1]), **f)  # noqa: E731
        dWD, dWE = torch.empty_like(WD), torch.empty_like(WE)
        dbD, dbE = torch.empty(WD.shape[0], **f), torch.empty(WE.shape[0], **f)
        dxv, dxp = torch.empty_like(xv), torch.empty_like(xp)
        _native.gvec_multi_bwd([(dXRv, xv, None, None, WD, dWD, dbD, None, None, part(WD)),
                                (dXRp, xp, None, None, WE, dWE, dbE, None, None, part(WE))],
                               [(0, 1, None, dxv), (1, 1, None, dxp)], 0.0)
        dW = [torch.empty_like(w) for w in (WA, WB, WC)]
        dbB, dbC = torch.empty(WB.shape[0], **f), torch.empty(WC.shape[0], **f)
        dln = [torch.empty_like(t) for t in (gA, bA, gB, bB, gC, bC)]
        dg = torch.empty_like(g1)
        _native.gvec_multi_bwd([(dsg, g1, gA, bA, WA, dW[0], None, dln[0], dln[1], part(WA)),
                                (dxv, g1, gB, bB, WB, dW[1], dbB, dln[2], dln[3], part(WB)),
                                (dxp, g1, gC, bC, WC, dW[2], dbC, dln[4], dln[5], part(WC))],
                               [(0, 3, dres, dg)], ctx.eps)
        return (dg.view(ctx.g_shape), dln[0], dln[1], dW[0], dln[2], dln[3], dW[1], dbB, dln[4], dln[5], dW[2], dbC,
                dWD, dbD, dWE, dbE, None)


def global_hub_params(pfu, nvsg):
    """GlobalHubFn parameters for this block's projection-feature update (pfu) and the next block's
    ViewAndScenePoint2Global (nvsg), or None when the shapes are not the fused ones."""
    if pfu is None or nvsg is None or not pfu.normalize_global_features or not nvsg.stateful:
        return None
    lnA, linA = pfu.global_norm_layer, pfu.lin_global
    G = linA.in_features
    seqs = (getattr(nvsg, "norm_and_proj_global2view", None), getattr(nvsg, "norm_and_proj_global2scenepoint", None))
    if any(q is None or len(q) != 3 or not isinstance(q[0], LayerNorm) or not isinstance(q[2], Linear) for q in seqs):
        return None
    (lnB, _, linB), (lnC, _, linC) = seqs
    linD, linE = nvsg.graph_conv_view2global.lin_r, nvsg.graph_conv_scenepoint2global.lin_r
    ok = (G % 64 == 0 and G <= GVEC_MAX_K and linA.bias is None and all(
        ln.weight is not None and ln.bias is not None and tuple(ln.normalized_shape) == (G,) and ln.eps == lnA.eps
        for ln in (lnA, lnB, lnC)) and linB.in_features == G and linC.in_features == G
        and linB.bias is not None and linC.bias is not None
        and linD.in_features == linB.out_features and linE.in_features == linC.out_features
        and linD.bias is not None and linE.bias is not None
        and all(n % 64 == 0 and n <= GVEC_MAX_K for n in (linD.in_features, linE.in_features)))
    if not ok:
        return None
    return (lnA.weight, lnA.bias, linA.weight, lnB.weight, lnB.bias, linB.weight, linB.bias, lnC.weight, lnC.bias,
            linC.weight, linC.bias, linD.weight, linD.bias, linE.weight, linE.bias, lnA.eps)


_GC_W = ("W1", "b1", "gM", "bM", "W2", "b2", "gA", "bA", "WA", "gB", "bB", "WB", "bWB", "gC", "bC", "WC", "bWC",
         "WD", "bD", "WE", "bE")
GCHAIN_MAX = 2048


_SHADOWS = {}  # id(weight) -> (weakref(weight), bf16 shadow, weight version, weight storage)


def weight_shadow(w):
    """w's bf16 shadow (BASELINE config 5: the global chain's GEMVs stream bf16 weights): re-rounded
    when w changed since its last use (version counter or storage).  A captured step's replays skip
    that check: call refresh_weight_shadows() after each optimizer step (GraphAttnSfMNet's
    refresh_weight_shadows)."""
    e = _SHADOWS.get(id(w))
    if e is not None and e[0]() is w:
        _, sh, ver, ptr = e
        if ver == w._version and ptr == w.data_ptr():
            return sh
    else:
        sh = torch.empty(w.shape, dtype=torch.bfloat16, device=w.device)
    with torch.no_grad():
        sh.copy_(w)
    _SHADOWS[id(w)] = (weakref.ref(w), sh, w._version, w.data_ptr())
    return sh


def refresh_weight_shadows():
    """Re-round every live bf16 shadow from its weight (after an optimizer step)."""
    with torch.no_grad():
        for k, (ref, sh, _, _) in list(_SHADOWS.items()):
            w = ref()
            if w is None:
                del _SHADOWS[k]
                continue
            sh.copy_(w)
            _SHADOWS[k] = (ref, sh, w._version, w.data_ptr())


class GlobalChainFn(torch.autograd.Function):
    """A block's whole global-node chain on ONE row (csrc/global_chain.hip), four launches each way:
    ViewAndScenePoint2Global's tail (layers.py:527-528, 590-603) and every consumer of its output g
    -- lin_global of the block's projection update (layers.py:928-935) and, when the next block has
    a global update, its norm_and_proj_global2view / _global2scenepoint (layers.py:497-520) and the
    two lin_r rows of its global convs.  Replaces the linear_res / ln_relu_linear GlobalLinearFns
    and GlobalHubFn (12 backward launches per block, each GEMV followed by a one-workgroup finish).

    apply(xcat [R, Kc], prev [R, G] or None, *weights (_GC_W order; the hub's B..E None for the last
    block), eps_m, eps_h, bf16) -> (g, SG, XRv, XRp), or (g, SG) without the hub, each [R, .].  R <= 7
    rows: a union batch's global nodes (one per scene), every weight streamed once for all of them.
    bf16: the GEMVs read the weights' bf16 shadows (weight_shadow; BASELINE config 5), fp32
    accumulation and gradients."""

    @staticmethod
    def forward(ctx, xcat, prev, *args):
        from . import _native
        ws, eps_m, eps_h, bf16 = args[:-3], args[-3], args[-2], args[-1]
        w = {k: (t.contiguous() if t is not None else None) for k, t in zip(_GC_W, ws)}
        sh = {k: weight_shadow(w[k]) for k in _native._GC_SHADOW if w[k] is not None} if bf16 else None
        R = xcat.shape[0]
        c = _native.gchain_struct(w, eps_m, eps_h, sh, rows=R)
        hub = w["WB"] is not None
        f = dict(dtype=torch.float32, device=xcat.device)
        x1c = xcat.contiguous()
        pv = prev.reshape(R, -1).contiguous() if prev is not None else None
        G = c.G
        x1, g, sg = torch.empty(R, G, **f), torch.empty(R, G, **f), torch.empty(R, c.NA, **f)
        xv = xp = xrv = xrp = None
        if hub:
            xv, xp, xrv, xrp = (torch.empty(R, n, **f) for n in (c.NB, c.NC, c.ND, c.NE))
        _native.gchain_fwd(c, x1c, pv, x1, g, sg, xv, xp, xrv, xrp)
        ctx.save_for_backward(x1c, x1, g, xv, xp, *(w[k] for k in _GC_W))
        ctx.eps = (eps_m, eps_h)
        ctx.shadows = sh
        ctx.hub, ctx.has_prev = hub, prev is not None
        ctx.shapes = (xcat.shape, prev.shape if prev is not None else None)
        ctx.set_materialize_grads(False)
        if hub:
            return g, sg, xrv, xrp
        return g, sg

    @staticmethod
    def backward(ctx, *grads):
        from . import _native
        x1c, x1, g, xv, xp, *wl = ctx.saved_tensors
        w = dict(zip(_GC_W, wl))
        R = g.shape[0]
        c = _native.gchain_struct(w, *ctx.eps, ctx.shadows, rows=R)
        f = dict(dtype=torch.float32, device=g.device)
        row = lambda t, n: t.reshape(R, n).contiguous() if t is not None else torch.zeros(R, n, **f)  # noqa: E731
        dskip = grads[0].reshape(R, -1).contiguous() if grads[0] is not None else None
        dsg = row(grads[1], c.NA)
        dxrv = dxrp = None
        if ctx.hub:
            dxrv, dxrp = row(grads[2], c.ND), row(grads[3], c.NE)
        d = {"d" + k: (torch.empty_like(t) if t is not None else None) for k, t in w.items()}
        dxcat = torch.empty(R, c.Kc, **f)
        dprev = torch.empty(R, c.G, **f) if ctx.has_prev else None
        _native.gchain_bwd(c, x1c, x1, g, xv, xp, dskip, dsg, dxrv, dxrp, dxcat, dprev, d)
        xs, ps = ctx.shapes
        return (dxcat.view(xs), dprev.view(ps) if dprev is not None else None,
                *(d["d" + k] for k in _GC_W), None, None, None)


def _ln_of(ln, G):
    return (isinstance(ln, LayerNorm) and tuple(ln.normalized_shape) == (G,) and ln.weight is not None
            and ln.bias is not None)


def chain_params(vsg, pfu, nvsg):
    """(weights in _GC_W order, eps_m, eps_h) of GlobalChainFn for ViewAndScenePoint2Global vsg's tail
    plus the consumers of its output: pfu's lin_global and, unless nvsg is None (the last block),
    the next block's global update nvsg; None when the shapes are not the fused kernels'."""
    if not hasattr(vsg, "proj_view_and_scenepoint2global") or not vsg.use_norm_pre_mlp or len(vsg.mlp) != 1:
        return None
    p1, lnM, l2 = vsg.proj_view_and_scenepoint2global, vsg.norm_pre_mlp, vsg.mlp[0]
    G, Kc = p1.out_features, p1.in_features
    fit = lambda n: n % 32 == 0 and 0 < n <= GCHAIN_MAX  # noqa: E731
    if not (fit(G) and fit(Kc) and p1.bias is not None and isinstance(l2, Linear) and l2.in_features == G
            and l2.out_features == G and l2.bias is not None and _ln_of(lnM, G)):
        return None
    if pfu is None or not pfu.normalize_global_features:
        return None
    lnA, linA = pfu.global_norm_layer, pfu.lin_global
    if not (_ln_of(lnA, G) and linA.bias is None and linA.in_features == G and linA.out_features <= GCHAIN_MAX):
        return None
    w = dict(W1=p1.weight, b1=p1.bias, gM=lnM.weight, bM=lnM.bias, W2=l2.weight, b2=l2.bias, gA=lnA.weight,
             bA=lnA.bias, WA=linA.weight)
    if nvsg is not None:
        hp = global_hub_params(pfu, nvsg)
        if hp is None:
            return None
        _, _, _, gB, bB, WB, bWB, gC, bC, WC, bWC, WD, bD, WE, bE, _ = hp
        if not (fit(WB.shape[0]) and fit(WC.shape[0]) and WD.shape[0] <= GCHAIN_MAX and WE.shape[0] <= GCHAIN_MAX):
            return None
        w.update(gB=gB, bB=bB, WB=WB, bWB=bWB, gC=gC, bC=bC, WC=WC, bWC=bWC, WD=WD, bD=bD, WE=WE, bE=bE)
    return tuple(w.get(k) for k in _GC_W), lnM.eps, lnA.eps


def global_chain(x, prev, params, bf16=False):
    """GlobalChainFn on the rows x [R, Kc] (prev [R, G] or None; R <= 7: one per scene of a union batch)
    when they fit, else None."""
    from . import _native
    if not (x.is_cuda and x.dim() == 2 and 1 <= x.shape[0] <= _native.GCHAIN_MAX_ROWS and x.dtype == torch.float32):
        return None
    if prev is not None and not (prev.numel() == x.shape[0] * params[0][0].shape[0] and prev.is_cuda):
        return None
    ws, eps_m, eps_h = params
    return GlobalChainFn.apply(x, prev, *ws, eps_m, eps_h, bool(bf16))


def _gvec_ok(x, k):
    return (x.is_cuda and x.dim() == 2 and x.shape[0] == 1 and x.dtype == torch.float32 and k % 64 == 0
            and k <= GVEC_MAX_K)


def linear(x, lin):
    if _gvec_ok(x, lin.in_features):
        return GlobalLinearFn.apply(x, None, None, lin.weight, lin.bias, None, 0.0, False)
    if (x.is_cuda and x.dim() == 2 and x.shape[0] > 0 and x.dtype == torch.float32 and lin.weight.dtype == x.dtype
            and torch.is_grad_enabled()):
        return RowLinearFn.apply(x, lin.weight, lin.bias)
    return F.linear(x, lin.weight, lin.bias)


def linear_res(x, lin, res):
    """lin(x) + res (res may be None)."""
    if _gvec_ok(x, lin.in_features) and (res is None or res.numel() == lin.out_features):
        return GlobalLinearFn.apply(x, None, None, lin.weight, lin.bias, res, 0.0, False)
    y = linear(x, lin)
    return y if res is None else res + y


# Row counts up to which a device LayerNorm over [rows, D] takes SmallLayerNormFn: there torch's
# backward reduces gamma / beta with a few-workgroup kernel (GammaBetaBackwardSimple: 41 us for
# 125 x 1024 on the rank-0-of-8 proxy's camera shard; 5-6 us per pass at 1000 rows)
SMALL_LN_ROWS = 512


class SmallLayerNormFn(torch.autograd.Function):
    """F.layer_norm whose backward takes dx from aten's row kernel and reduces gamma / beta as
    one [rows, 2D] partial matrix [dy xhat | dy] through param_colsum (batched with the step's
    other parameter sums at the end of the backward pass)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        D = x.shape[-1]
        y, mean, rstd = torch.native_layer_norm(x, [D], w, b, eps)
        ctx.save_for_backward(x, mean, rstd, w, b)
        from . import _native
        ctx.defer = _native.defer_token(w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _native
        x, mean, rstd, w, b = ctx.saved_tensors
        D = x.shape[-1]
        dy = dy.contiguous()
        dx = torch.ops.aten.native_layer_norm_backward(dy, x, [D], mean, rstd, w, b, [True, False, False])[0]
        part = torch.empty((x.shape[0], 2 * D), dtype=dy.dtype, device=dy.device)
        torch.sub(x, mean, out=part[:, :D])
        part[:, :D].mul_(rstd).mul_(dy)
        part[:, D:].copy_(dy)
        tot = _native.param_colsum(part, ctx.defer)
        # views of the (possibly deferred) sum: AccumulateGrad adopts a view, it would copy the
        # pending sum tensor itself before it is filled
        return dx, tot[:D], tot[D:], None


def layer_norm(x, ln):
    if (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and 0 < x.shape[0] <= SMALL_LN_ROWS
            and ln.weight is not None and ln.bias is not None and torch.is_grad_enabled()
            and x.stride(1) == 1 and (x.requires_grad or ln.weight.requires_grad)):
        return SmallLayerNormFn.apply(x, ln.weight, ln.bias, ln.eps)
    return F.layer_norm(x, ln.normalized_shape, ln.weight, ln.bias, ln.eps)


NODE_WIDTH = 64  # n_feat_scenepoint of every GASFM conf: the width node_block.hip is built for


class NodeLnLinearFn(torch.autograd.Function):
    """y = W relu(LN(x)) + b (+ x): one HIP kernel each way (csrc/node_block.hip).

    Backward recomputes the LayerNorm statistics from x and returns dx plus the weight,
    bias, gamma and beta gradients reduced deterministically (per-workgroup partials ->
    gasfm_colsum)."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, W, b, eps, residual):
        from . import _native
        x = x.contiguous()
        W = W.contiguous()
        y = torch.empty((x.shape[0], W.shape[0]), dtype=torch.float32, device=x.device)
        _native.node_ln_linear_fwd(x, ln_w, ln_b, eps, W, b, residual, y)
        ctx.save_for_backward(x, ln_w, ln_b, W)
        ctx.eps, ctx.residual, ctx.has_b = eps, residual, b is not None
        ctx.defer = _native.defer_token(ln_w, ln_b, W, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _native
        x, ln_w, ln_b, W = ctx.saved_tensors
        n_out, n_in = W.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        rows = _native.node_part_rows(x.shape[0], n_out, ctx.residual)
        part = torch.empty((rows, n_out * n_in + n_out + 2 * n_in), dtype=torch.float32, device=x.device)
        _native.node_ln_linear_bwd(dy, x, ln_w, ln_b, ctx.eps, W, ctx.residual, dx, part)
        tot = _native.param_colsum(part, ctx.defer)
        o = n_out * n_in
        dW = tot[:o].view(n_out, n_in)
        db = tot[o:o + n_out] if ctx.has_b else None
        dg = tot[o + n_out:o + n_out + n_in]
        dbeta = tot[o + n_out + n_in:]
        return dx, dg, dbeta, dW, db, None, None


def _node_fusable(x, ln, lin):
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and x.shape[1] == NODE_WIDTH
            and tuple(ln.normalized_shape) == (NODE_WIDTH,) and ln.weight is not None and ln.bias is not None
            and lin.in_features == NODE_WIDTH and lin.out_features in (32, 64))


def _gvec_ln_ok(x, ln, lin, residual):
    return (_gvec_ok(x, lin.in_features) and ln.weight is not None and ln.bias is not None
            and tuple(ln.normalized_shape) == (lin.in_features,)
            and (not residual or lin.out_features == lin.in_features))


def ln_relu_linear(x, ln, lin, residual=False):
    """lin(relu(ln(x))) (+ x when residual): the fused point-node kernel for 64-wide rows, the
    global-vector kernel for a single row."""
    if _node_fusable(x, ln, lin) and (not residual or lin.out_features == NODE_WIDTH):
        return NodeLnLinearFn.apply(x, ln.weight, ln.bias, lin.weight, lin.bias, ln.eps, residual)
    if _gvec_ln_ok(x, ln, lin, residual):
        return GlobalLinearFn.apply(x, ln.weight, ln.bias, lin.weight, lin.bias, None, ln.eps, residual)
    y = linear(F.relu(layer_norm(x, ln)), lin)
    return x + y if residual else y


def sequential(seq, x):
    """Run a Sequential of Linear / LayerNorm / ReLU with the row-aware linear; a
    LayerNorm, ReLU, Linear run on 64-wide point rows or on the single global row goes
    through a fused kernel."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        mod = mods[i]
        if (isinstance(mod, LayerNorm) and i + 2 < len(mods) and isinstance(mods[i + 1], ReLU)
                and isinstance(mods[i + 2], Linear)
                and (_node_fusable(x, mod, mods[i + 2]) or _gvec_ln_ok(x, mod, mods[i + 2], False))):
            x = ln_relu_linear(x, mod, mods[i + 2])
            i += 3
            continue
        i += 1
        if isinstance(mod, Linear):
            x = linear(x, mod)
        elif isinstance(mod, LayerNorm):
            x = layer_norm(x, mod)
        elif isinstance(mod, ReLU):
            x = F.relu(x)
        else:
            x = mod(x)
    return x
