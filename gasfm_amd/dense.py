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
    (split-K slices, camera rows); torch's reduction for tall ones (200k point rows), where
    colsum's <= 64 row blocks per column chunk would leave the chip idle."""
    if a.shape[0] > 4096:
        return a.sum(0)
    from . import _native
    return _native.colsum(a.contiguous())


def splitk_wgrad(dy, x):
    R, M = dy.shape
    N = x.shape[1]
    if R < 16384 and M * N > 262144:
        return dy.T @ x  # camera 1024x1024 weights: already 256 output tiles, no split
    B = max(1, min(_MAX_SLICES, R // _MIN_CHUNK))
    R0 = (R // B) * B
    dW = _colsum(torch.bmm(dy[:R0].reshape(B, R0 // B, M).transpose(1, 2), x[:R0].reshape(B, R0 // B, N))
                 .reshape(B, M * N)).view(M, N)
    if R0 < R:
        dW = dW + dy[R0:].T @ x[R0:]
    return dW


class RowLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return F.linear(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy @ W if ctx.needs_input_grad[0] else None
        dW = splitk_wgrad(dy, x.contiguous()) if ctx.needs_input_grad[1] else None
        db = _colsum(dy) if ctx.has_b and ctx.needs_input_grad[2] else None
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


def _gvec_ok(x, k):
    return (x.is_cuda and x.dim() == 2 and x.shape[0] == 1 and x.dtype == torch.float32 and k % 64 == 0
            and k <= GVEC_MAX_K)


def linear(x, lin):
    if _gvec_ok(x, lin.in_features):
        return GlobalLinearFn.apply(x, None, None, lin.weight, lin.bias, None, 0.0, False)
    if x.is_cuda and x.dim() == 2 and x.shape[0] >= SPLITK_MIN_ROWS and torch.is_grad_enabled():
        return RowLinearFn.apply(x, lin.weight, lin.bias)
    return F.linear(x, lin.weight, lin.bias)


def linear_res(x, lin, res):
    """lin(x) + res (res may be None)."""
    if _gvec_ok(x, lin.in_features) and (res is None or res.numel() == lin.out_features):
        return GlobalLinearFn.apply(x, None, None, lin.weight, lin.bias, res, 0.0, False)
    y = linear(x, lin)
    return y if res is None else res + y


def layer_norm(x, ln):
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
        tot = _native.colsum(part)
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
