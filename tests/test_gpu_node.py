"""Point-node LayerNorm -> ReLU -> Linear (-> + x) kernels (csrc/node_block.hip) vs fp64 torch.

The op is the composition the reference runs with aten modules (layers.py:48-56, 449-456,
928-935); the fp64 evaluation of that composition is the reference here.  Tolerance: fp32
outputs within 2e-5 * max|ref| + 1e-5 elementwise; gradients normwise 1e-4 (LayerNorm backward
in fp32 over 64 columns, weight gradients reduced over up to 200k rows).
"""
import pytest
import torch
import torch.nn.functional as F

from gasfm_amd import dense

pytestmark = pytest.mark.gpu


def _ref(x, g, b, W, bias, eps, residual):
    y = F.linear(F.relu(F.layer_norm(x, (x.shape[1],), g, b, eps)), W, bias)
    return x + y if residual else y


@pytest.mark.parametrize("N", [0, 1, 15, 16, 17, 1000, 70_001])
@pytest.mark.parametrize("n_out,residual,has_bias", [(32, False, True), (32, False, False), (64, True, True),
                                                      (64, False, True)])
def test_node_ln_linear_matches_fp64(device, N, n_out, residual, has_bias):
    g = torch.Generator().manual_seed(N * 7 + n_out + residual)
    x = torch.randn(N, 64, generator=g, dtype=torch.float64) * 2 + 0.5
    gam = 1 + 0.3 * torch.randn(64, generator=g, dtype=torch.float64)
    bet = 0.2 * torch.randn(64, generator=g, dtype=torch.float64)
    W = torch.randn(n_out, 64, generator=g, dtype=torch.float64) / 8
    bias = torch.randn(n_out, generator=g, dtype=torch.float64) if has_bias else None
    dy = torch.randn(N, n_out, generator=g, dtype=torch.float64)
    ins64 = [t.clone().requires_grad_(True) if t is not None else None for t in (x, gam, bet, W, bias)]
    y64 = _ref(*ins64[:4], ins64[4], 1e-5, residual)
    y64.backward(dy)
    ins = [t.float().to(device).requires_grad_(True) if t is not None else None for t in (x, gam, bet, W, bias)]
    y = dense.NodeLnLinearFn.apply(ins[0], ins[1], ins[2], ins[3], ins[4], 1e-5, residual)
    y.backward(dy.float().to(device))
    if N == 0:
        assert y.shape == (0, n_out)
        return
    scale = y64.abs().max().item()
    torch.testing.assert_close(y.double().cpu(), y64.detach(), rtol=0, atol=2e-5 * scale + 1e-5)
    for name, a, r in zip(("x", "gamma", "beta", "W", "bias"), ins, ins64):
        if a is None:
            continue
        ga, gr = a.grad.double().cpu(), r.grad
        err = (ga - gr).norm().item()
        assert err <= 1e-4 * gr.norm().item() + 1e-6, f"{name}: {err:.3e} vs |ref| {gr.norm().item():.3e}"


def test_node_ln_linear_deterministic(device):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(50_000, 64, generator=g).to(device).requires_grad_(True)
    ln = torch.nn.LayerNorm(64).to(device)
    lin = torch.nn.Linear(64, 64).to(device)
    outs = []
    for _ in range(2):
        x.grad = None
        lin.zero_grad()
        ln.zero_grad()
        y = dense.ln_relu_linear(x, ln, lin, residual=True)
        y.square().sum().backward()
        outs.append([y.detach().clone(), x.grad.clone(), lin.weight.grad.clone(), ln.weight.grad.clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_node_dispatch_uses_kernel_for_point_rows(device):
    """sequential() routes LayerNorm, ReLU, Linear on 64-wide CUDA rows to the fused kernel."""
    seq = torch.nn.Sequential(torch.nn.LayerNorm(64), torch.nn.ReLU(), torch.nn.Linear(64, 32)).to(device)
    x = torch.randn(100, 64, device=device, requires_grad=True)
    y = dense.sequential(seq, x)
    assert type(y.grad_fn).__name__ == "NodeLnLinearFnBackward"
    torch.testing.assert_close(y, seq(x), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("N,D", [(1, 1024), (125, 1024), (512, 64), (300, 4)])
def test_small_layer_norm_matches_fp64(device, N, D):
    """dense.layer_norm on few rows (SmallLayerNormFn: aten's dx, gamma / beta through
    param_colsum) vs fp64 F.layer_norm; the same tolerances as above."""
    g = torch.Generator().manual_seed(N + D)
    x = torch.randn(N, D, generator=g, dtype=torch.float64) * 2 + 0.5
    ln = torch.nn.LayerNorm(D).double()
    with torch.no_grad():
        ln.weight.copy_(1 + 0.3 * torch.randn(D, generator=g, dtype=torch.float64))
        ln.bias.copy_(0.2 * torch.randn(D, generator=g, dtype=torch.float64))
    dy = torch.randn(N, D, generator=g, dtype=torch.float64)
    x64 = x.clone().requires_grad_(True)
    y64 = F.layer_norm(x64, (D,), ln.weight, ln.bias, ln.eps)
    y64.backward(dy)
    ln32 = torch.nn.LayerNorm(D).to(device)
    with torch.no_grad():
        ln32.weight.copy_(ln.weight.float())
        ln32.bias.copy_(ln.bias.float())
    x32 = x.float().to(device).requires_grad_(True)
    y = dense.layer_norm(x32, ln32)
    assert "SmallLayerNorm" in type(y.grad_fn).__name__
    y.backward(dy.float().to(device))
    torch.testing.assert_close(y.double().cpu(), y64.detach(), rtol=0, atol=2e-5 * y64.abs().max().item() + 1e-5)
    for got, ref, nm in ((x32.grad, x64.grad, "dx"), (ln32.weight.grad, ln.weight.grad, "dgamma"),
                         (ln32.bias.grad, ln.bias.grad, "dbeta")):
        err = (got.double().cpu() - ref).norm().item()
        assert err <= 1e-4 * ref.norm().item() + 1e-6, f"{nm}: {err:.3e} vs |ref| {ref.norm().item():.3e}"
