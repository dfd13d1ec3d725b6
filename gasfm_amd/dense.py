"""Dense per-node layers (point rows: n ~ 200k) with a split-K weight gradient.

torch's Linear backward computes dW = dY^T X as ONE GEMM with K = rows; for the
GASFM point layers (M, N <= 64, K = 200k) hipBLASLt then runs one or two
workgroups (measured 0.45-0.53 ms per call on MI355X, ~40 ms per training
step).  ``linear`` keeps torch's forward / input-gradient GEMMs (MFMA through
hipBLASLt, good shapes) and computes the weight gradient as a batched GEMM over
row chunks followed by a sum (split-K), which fills the chip.
Camera / global rows (<= a few thousand) go through plain torch.
"""
import torch
import torch.nn.functional as F
from torch.nn import LayerNorm, Linear, ReLU, Sequential

SPLITK_MIN_ROWS = 16384
_CHUNK = 2048


def splitk_wgrad(dy, x):
    R, M = dy.shape
    N = x.shape[1]
    B = max(1, min(256, R // _CHUNK))
    R0 = (R // B) * B
    dW = torch.bmm(dy[:R0].reshape(B, R0 // B, M).transpose(1, 2), x[:R0].reshape(B, R0 // B, N)).sum(0)
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
        db = dy.sum(0) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dW, db


def linear(x, lin):
    if x.is_cuda and x.dim() == 2 and x.shape[0] >= SPLITK_MIN_ROWS and torch.is_grad_enabled():
        return RowLinearFn.apply(x, lin.weight, lin.bias)
    return F.linear(x, lin.weight, lin.bias)


def layer_norm(x, ln):
    return F.layer_norm(x, ln.normalized_shape, ln.weight, ln.bias, ln.eps)


def sequential(seq, x):
    """Run a Sequential of Linear / LayerNorm / ReLU with the row-aware linear."""
    for mod in seq:
        if isinstance(mod, Linear):
            x = linear(x, mod)
        elif isinstance(mod, LayerNorm):
            x = layer_norm(x, mod)
        elif isinstance(mod, ReLU):
            x = F.relu(x)
        else:
            x = mod(x)
    return x
