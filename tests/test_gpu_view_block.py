"""Fused camera-side tail / hub (csrc/view_block.hip + hipBLASLt GEMMs; at m <= 256 rows and D in
{256, 512, 1024} csrc/view_chain.hip, the GEMMs with the view kernels fused in) vs the fp64 torch
composition of the reference's ops (Proj2View.forward layers.py:345-360; lin_view(relu(
view_norm_layer(v))) :928-935; the next block's lin_r(norm_and_proj_view2proj(v)) :331;
graph_conv_view2global.lin_l).  Tolerance: outputs 2e-5 * max|ref| + 1e-5 (GEMMs with K up to
1024 in fp32); gradients normwise 1e-4.
"""
import pytest
import torch
import torch.nn.functional as F

from gasfm_amd import view_block

pytestmark = pytest.mark.gpu
EPS = 1e-5


def _rnd(g, *shape, scale=1.0, shift=0.0):
    return torch.randn(*shape, generator=g, dtype=torch.float64) * scale + shift


def _check(outs, refs, names):
    for name, o, r in zip(names, outs, refs):
        torch.testing.assert_close(o.double().cpu(), r.detach(), rtol=0, atol=2e-5 * r.abs().max().item() + 1e-5,
                                   msg=name)


def _check_grads(names, got, ref):
    for name, a, r in zip(names, got, ref):
        if r is None:
            continue
        ga, gr = a.grad.double().cpu(), r.grad
        err = (ga - gr).norm().item()
        assert err <= 1e-4 * gr.norm().item() + 1e-6, f"{name}: {err:.3e} vs |ref| {gr.norm().item():.3e}"


@pytest.mark.parametrize("m", [1, 17, 125, 256, 1000])
@pytest.mark.parametrize("D", [64, 192, 256, 1024])
@pytest.mark.parametrize("with_prev", [True, False])
def test_view_tail_matches_fp64(device, m, D, with_prev):
    g = torch.Generator().manual_seed(m + D + with_prev)
    ins = [_rnd(g, m, D, scale=2, shift=0.1) if with_prev else None, _rnd(g, m, 32), _rnd(g, D, 32, scale=0.2),
           _rnd(g, D, scale=0.1), _rnd(g, D, scale=0.3, shift=1), _rnd(g, D, scale=0.2),
           _rnd(g, D, D, scale=D ** -0.5), _rnd(g, D, scale=0.1)]
    dout = _rnd(g, m, D)
    ref = [t.clone().requires_grad_(True) if t is not None else None for t in ins]
    prev, agg, Wp, bp, gm, bt, Wm, bm = ref
    x = F.linear(agg, Wp, bp) + (prev if prev is not None else 0)
    y64 = x + F.linear(F.relu(F.layer_norm(x, (D,), gm, bt, EPS)), Wm, bm)
    y64.backward(dout)
    got = [t.float().to(device).requires_grad_(True) if t is not None else None for t in ins]
    y = view_block.ViewTailFn.apply(*got, EPS)
    y.backward(dout.float().to(device))
    _check([y], [y64], ["view"])
    _check_grads(("prev", "agg", "Wp", "bp", "gamma", "beta", "Wm", "bm"), got, ref)


@pytest.mark.parametrize("m", [1, 17, 125, 256, 1000])
@pytest.mark.parametrize("D", [64, 192, 256, 1024])
@pytest.mark.parametrize("with_skip", [True, False])
@pytest.mark.parametrize("packed", [False, True])
def test_view_hub_matches_fp64(device, m, D, with_skip, packed):
    g = torch.Generator().manual_seed(7 * m + D + with_skip)
    ins = [_rnd(g, m, D, scale=1.5, shift=-0.1), _rnd(g, D, scale=0.3, shift=1), _rnd(g, D, scale=0.2),
           _rnd(g, 32, D, scale=D ** -0.5), _rnd(g, D, D, scale=D ** -0.5), _rnd(g, D, scale=0.1),
           _rnd(g, D, scale=0.3, shift=1), _rnd(g, D, scale=0.2), _rnd(g, 32, D, scale=D ** -0.5),
           _rnd(g, 32, scale=0.1), _rnd(g, 32, 32, scale=0.18), _rnd(g, 32, scale=0.1)]
    grads = [_rnd(g, m, D) if with_skip else None, _rnd(g, m, 32), _rnd(g, m, D), _rnd(g, m, 32)]
    ref = [t.clone().requires_grad_(True) for t in ins]
    v, gC, bC, Wv, Wl, bl, gA, bA, Wa, ba, Wr, br = ref
    outs64 = (v, F.linear(F.relu(F.layer_norm(v, (D,), gC, bC, EPS)), Wv), F.linear(v, Wl, bl),
              F.linear(F.linear(F.relu(F.layer_norm(v, (D,), gA, bA, EPS)), Wa, ba), Wr, br))
    torch.autograd.backward([o for o, d in zip(outs64, grads) if d is not None], [d for d in grads if d is not None])
    got = [t.float().to(device).requires_grad_(True) for t in ins]
    outs = view_block.ViewHubFn.apply(*got, EPS, False, packed)
    _check(outs, outs64, ("skip", "SV", "XL", "XR"))
    torch.autograd.backward([o for o, d in zip(outs, grads) if d is not None],
                            [d.float().to(device) for d in grads if d is not None])
    _check_grads(("v", "gC", "bC", "Wv", "Wl", "bl", "gA", "bA", "Wa", "ba", "Wr", "br"), got, ref)


def test_view_chain_dispatch(device):
    """Small row counts with a supported width take the fused view_chain kernels (ctx.chain), the
    1000-row config-4 camera side the view kernels + hipBLASLt; the ABI predicate agrees."""
    from gasfm_amd import _native
    assert _native.view_chain_ok(125, 1024) and _native.view_chain_ok(256, 512)
    assert not _native.view_chain_ok(257, 1024) and not _native.view_chain_ok(125, 192)
    for m, want in ((125, True), (1000, False)):
        x = torch.randn(m, 32, device=device, requires_grad=True)
        W = [torch.randn(*s, device=device) * 0.05 for s in ((1024, 32), (1024,), (1024,), (1024,), (1024, 1024),
                                                              (1024,))]
        y = view_block.ViewTailFn.apply(None, x, *W, EPS)
        assert y.grad_fn._forward_cls is view_block.ViewTailFn
        # the Function's ctx is the grad_fn node
        assert y.grad_fn.chain == (want and view_block.VIEW_CHAIN)
