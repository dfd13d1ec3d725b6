"""Embed2Fn (csrc/embed.hip): the input embedding P = values W^T + b, the Linear(2, 2) of the
reference's EmbeddingLayer (code/models/layers.py:992-1015, graph_attn_sfm.py:53), against fp64.

Forward: two fmas per output, so within 2 fp32 roundings of |W||x| + |b| per element.  Weight
and bias gradients are sums over E rows: normwise within 1e-5 of fp64 (fp32 partial sums of <=
a few thousand terms each, then an ordered column sum).  Bitwise repeatable."""
import pytest
import torch

from gasfm_amd.model import Embed2Fn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("E", [1, 2, 7, 1000, 4_001_638])
def test_forward_backward(device, E):
    g = torch.Generator(device="cpu").manual_seed(E)
    x = torch.randn(E, 2, generator=g).to(device)
    W = torch.randn(2, 2, generator=g).to(device).requires_grad_(True)
    b = torch.randn(2, generator=g).to(device).requires_grad_(True)
    dy = torch.randn(E, 2, generator=g).to(device)
    y = Embed2Fn.apply(x, W, b)
    y.backward(dy)
    x64, W64, b64, dy64 = x.double(), W.detach().double(), b.detach().double(), dy.double()
    ref = x64 @ W64.t() + b64
    bound = 2 * 2.0 ** -23 * (x64.abs() @ W64.abs().t() + b64.abs())
    assert bool(((y.double() - ref).abs() <= bound + 1e-30).all())
    dW_ref, db_ref = dy64.t() @ x64, dy64.sum(0)
    assert (W.grad.double() - dW_ref).norm() <= 1e-5 * dW_ref.norm() + 1e-6
    assert (b.grad.double() - db_ref).norm() <= 1e-5 * db_ref.norm() + 1e-6
    dW1, db1 = W.grad.clone(), b.grad.clone()
    W.grad = b.grad = None
    Embed2Fn.apply(x, W, b).backward(dy)
    assert torch.equal(W.grad, dW1) and torch.equal(b.grad, db1)


def test_empty(device):
    W = torch.randn(2, 2, device=device, requires_grad=True)
    b = torch.randn(2, device=device, requires_grad=True)
    y = Embed2Fn.apply(torch.zeros(0, 2, device=device), W, b)
    assert y.shape == (0, 2)
    y.sum().backward()
    assert float(W.grad.abs().sum()) == 0.0 and float(b.grad.abs().sum()) == 0.0
