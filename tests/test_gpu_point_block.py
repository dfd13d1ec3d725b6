"""Fused scene-point tail / hub (csrc/point_block.hip) vs the fp64 torch composition.

The composition is the reference's op sequence (Proj2ScenePoint.forward layers.py:438-454;
lin_scenepoint(relu(scenepoint_norm_layer(p))) :928-935; graph_conv_scenepoint2global.lin_l;
the next block's norm_and_proj_scenepoint2proj + lin_r), evaluated in fp64 with autograd.
Tolerance: outputs 2e-5 * max|ref| + 1e-5 elementwise; gradients normwise 1e-4 (fp32
LayerNorm backward over 64 columns, weight gradients reduced over up to 70k rows).
"""
import pytest
import torch
import torch.nn.functional as F

from gasfm_amd import point_block

pytestmark = pytest.mark.gpu
EPS = 1e-5


def _rnd(g, *shape, scale=1.0, shift=0.0):
    return torch.randn(*shape, generator=g, dtype=torch.float64) * scale + shift


def _close_grads(names, got, ref):
    for name, a, r in zip(names, got, ref):
        if r is None:
            continue
        ga, gr = a.grad.double().cpu(), r.grad
        err = (ga - gr).norm().item()
        assert err <= 1e-4 * gr.norm().item() + 1e-6, f"{name}: {err:.3e} vs |ref| {gr.norm().item():.3e}"


def _tail_ref(prev, agg, Wp, bp, g, b, Wm, bm):
    x = F.linear(agg, Wp, bp)
    if prev is not None:
        x = prev + x
    return x + F.linear(F.relu(F.layer_norm(x, (64,), g, b, EPS)), Wm, bm)


@pytest.mark.parametrize("N", [1, 15, 16, 17, 1000, 70_001])
@pytest.mark.parametrize("with_prev", [True, False])
def test_point_tail_matches_fp64(device, N, with_prev):
    g = torch.Generator().manual_seed(N + 11 * with_prev)
    ins = [_rnd(g, N, 64, scale=2, shift=0.3) if with_prev else None, _rnd(g, N, 32),
           _rnd(g, 64, 32, scale=0.2), _rnd(g, 64, scale=0.1), _rnd(g, 64, scale=0.3, shift=1), _rnd(g, 64, scale=0.2),
           _rnd(g, 64, 64, scale=0.125), _rnd(g, 64, scale=0.1)]
    dout = _rnd(g, N, 64)
    ref = [t.clone().requires_grad_(True) if t is not None else None for t in ins]
    y64 = _tail_ref(*ref)
    y64.backward(dout)
    got = [t.float().to(device).requires_grad_(True) if t is not None else None for t in ins]
    y = point_block.PointTailFn.apply(*got, EPS)
    y.backward(dout.float().to(device))
    torch.testing.assert_close(y.double().cpu(), y64.detach(), rtol=0, atol=2e-5 * y64.abs().max().item() + 1e-5)
    _close_grads(("prev", "agg", "Wp", "bp", "gamma", "beta", "Wm", "bm"), got, ref)


def _hub_ref(p, gA, bA, WA, WB, bB, gC, bC, WC, bWC, WD, bD):
    SA = F.linear(F.relu(F.layer_norm(p, (64,), gA, bA, EPS)), WA)
    XL = F.linear(p, WB, bB)
    XR = F.linear(F.linear(F.relu(F.layer_norm(p, (64,), gC, bC, EPS)), WC, bWC), WD, bD)
    return p, SA, XL, XR


@pytest.mark.parametrize("N", [1, 17, 1000, 70_001])
@pytest.mark.parametrize("with_skip", [True, False])
def test_point_hub_matches_fp64(device, N, with_skip):
    g = torch.Generator().manual_seed(3 * N + with_skip)
    ins = [_rnd(g, N, 64, scale=1.5, shift=-0.2), _rnd(g, 64, scale=0.3, shift=1), _rnd(g, 64, scale=0.2),
           _rnd(g, 32, 64, scale=0.125), _rnd(g, 64, 64, scale=0.125), _rnd(g, 64, scale=0.1),
           _rnd(g, 64, scale=0.3, shift=1), _rnd(g, 64, scale=0.2), _rnd(g, 32, 64, scale=0.125),
           _rnd(g, 32, scale=0.1), _rnd(g, 32, 32, scale=0.18), _rnd(g, 32, scale=0.1)]
    dsk, dSA, dXL, dXR = _rnd(g, N, 64), _rnd(g, N, 32), _rnd(g, N, 64), _rnd(g, N, 32)
    ref = [t.clone().requires_grad_(True) for t in ins]
    outs64 = _hub_ref(*ref)
    grads = [dsk if with_skip else None, dSA, dXL, dXR]
    torch.autograd.backward([o for o, d in zip(outs64, grads) if d is not None], [d for d in grads if d is not None])
    got = [t.float().to(device).requires_grad_(True) for t in ins]
    outs = point_block.PointHubFn.apply(*got, EPS)
    for name, o, r in zip(("skip", "SA", "XL", "XR"), outs, outs64):
        torch.testing.assert_close(o.double().cpu(), r.detach(), rtol=0, atol=2e-5 * r.abs().max().item() + 1e-5,
                                   msg=name)
    torch.autograd.backward([o for o, d in zip(outs, grads) if d is not None],
                            [d.float().to(device) for d in grads if d is not None])
    _close_grads(("p", "gA", "bA", "WA", "WB", "bB", "gC", "bC", "WC", "bWC", "WD", "bD"), got, ref)


def test_point_hub_deterministic(device):
    g = torch.Generator().manual_seed(5)
    ins = [_rnd(g, 50_000, 64).float().to(device).requires_grad_(True)] + [
        t.float().to(device).requires_grad_(True) for t in (
            1 + 0.1 * _rnd(g, 64), 0.1 * _rnd(g, 64), _rnd(g, 32, 64) / 8, _rnd(g, 64, 64) / 8, _rnd(g, 64),
            1 + 0.1 * _rnd(g, 64), 0.1 * _rnd(g, 64), _rnd(g, 32, 64) / 8, _rnd(g, 32), _rnd(g, 32, 32) / 6,
            _rnd(g, 32))]
    res = []
    for _ in range(2):
        for t in ins:
            t.grad = None
        outs = point_block.PointHubFn.apply(*ins, EPS)
        sum(o.square().sum() for o in outs).backward()
        res.append([t.grad.clone() for t in ins])
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N", [1, 17, 1000, 70_001])
@pytest.mark.parametrize("with_prev", [True, False])
def test_point_tail_hub_fused_bitwise(device, N, with_prev):
    """PointTailHubFn (one forward kernel, round 6) against PointTailFn then PointHubFn: the same tile
    bodies, so p / SA / XL / XR are bitwise equal, and the gradients -- the same backward kernels in the
    same order, the skip gradient entering the hub as dRes -- bitwise too; plus the fp64 composition."""
    g = torch.Generator().manual_seed(7 * N + with_prev)
    tail_in = [_rnd(g, N, 64, scale=2, shift=0.3) if with_prev else None, _rnd(g, N, 32),
               _rnd(g, 64, 32, scale=0.2), _rnd(g, 64, scale=0.1), _rnd(g, 64, scale=0.3, shift=1),
               _rnd(g, 64, scale=0.2), _rnd(g, 64, 64, scale=0.125), _rnd(g, 64, scale=0.1)]
    hub_in = [_rnd(g, 64, scale=0.3, shift=1), _rnd(g, 64, scale=0.2), _rnd(g, 32, 64, scale=0.125),
              _rnd(g, 64, 64, scale=0.125), _rnd(g, 64, scale=0.1), _rnd(g, 64, scale=0.3, shift=1),
              _rnd(g, 64, scale=0.2), _rnd(g, 32, 64, scale=0.125), _rnd(g, 32, scale=0.1),
              _rnd(g, 32, 32, scale=0.18), _rnd(g, 32, scale=0.1)]
    dp, dSA, dXL, dXR = _rnd(g, N, 64), _rnd(g, N, 32), _rnd(g, N, 64), _rnd(g, N, 32)
    dev = lambda ts: [t.float().to(device).requires_grad_(True) if t is not None else None for t in ts]  # noqa: E731
    # the two Functions
    t2, h2 = dev(tail_in), dev(hub_in)
    p2 = point_block.PointTailFn.apply(*t2, EPS)
    outs2 = point_block.PointHubFn.apply(p2, *h2, EPS)
    torch.autograd.backward(outs2, [d.float().to(device) for d in (dp, dSA, dXL, dXR)])
    # one kernel
    t1, h1 = dev(tail_in), dev(hub_in)
    outs1 = point_block.PointTailHubFn.apply(*t1, EPS, *h1, EPS)
    for name, a, b in zip(("p", "SA", "XL", "XR"), outs1, outs2):
        assert torch.equal(a, b), name
    torch.autograd.backward(outs1, [d.float().to(device) for d in (dp, dSA, dXL, dXR)])
    for name, a, b in zip(("prev", "agg", "Wp", "bp", "gamma", "beta", "Wm", "bm", "gA", "bA", "WA", "WB", "bB",
                           "gC", "bC", "WC", "bWC", "WD", "bD"), t1 + h1, t2 + h2):
        if a is None:
            continue
        assert torch.equal(a.grad, b.grad), name
    # and against the fp64 composition
    r_t = [t.clone().requires_grad_(True) if t is not None else None for t in tail_in]
    r_h = [t.clone().requires_grad_(True) for t in hub_in]
    outs64 = _hub_ref(_tail_ref(*r_t), *r_h)
    for name, o, r in zip(("p", "SA", "XL", "XR"), outs1, outs64):
        torch.testing.assert_close(o.double().cpu(), r.detach(), rtol=0, atol=5e-5 * r.abs().max().item() + 1e-5,
                                   msg=name)
    torch.autograd.backward(list(outs64), [dp, dSA, dXL, dXR])
    _close_grads(("prev", "agg", "Wp", "bp", "gamma", "beta", "Wm", "bm", "gA", "bA", "WA", "WB", "bB", "gC", "bC",
                  "WC", "bWC", "WD", "bD"), t1 + h1, r_t + r_h)
