"""gasfm_amd.optim.Adam (csrc/adam.hip: every tensor of a group in one launch) against torch.optim.Adam.

Same update (torch/optim/adam.py, amsgrad off): after 4 steps with fresh random gradients each step,
parameters and both moment buffers agree within rtol 2e-6, atol 1e-7 (the kernel multiplies by
1 / sqrt(1 - beta2^t) where torch divides; single-rounding fma in the moments).  Covers tensor sizes
that are not multiples of 4 or of the 4096-value chunk, weight decay on and off, and a gradient
tensor swapped between steps (the pointer table is rebuilt).
"""
import copy

import pytest
import torch

from gasfm_amd.optim import Adam

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_matches_torch(device, wd):
    gen = torch.Generator().manual_seed(5)
    shapes = [(2048, 1088), (2048,), (33,), (7, 5), (4096 * 3 + 1,), (1,)]
    ref = [torch.randn(s, generator=gen).to(device).requires_grad_(True) for s in shapes]
    got = [r.detach().clone().requires_grad_(True) for r in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    o_got = Adam(got, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    for it in range(4):
        for a, b in zip(ref, got):
            g = torch.randn(a.shape, generator=gen).to(device)
            a.grad = g.clone()
            b.grad = g.clone()  # a new gradient tensor every step: the table is rebuilt
        o_ref.step()
        o_got.step()
    for a, b in zip(ref, got):
        torch.testing.assert_close(b, a, rtol=2e-6, atol=1e-7)
        sa, sb = o_ref.state[a], o_got.state[b]
        torch.testing.assert_close(sb["exp_avg"], sa["exp_avg"], rtol=2e-6, atol=1e-7)
        torch.testing.assert_close(sb["exp_avg_sq"], sa["exp_avg_sq"], rtol=2e-6, atol=1e-7)
        assert int(sb["step"]) == 4


def test_adam_rejects_unsupported(device):
    p = torch.zeros(4, device=device, requires_grad=True)
    with pytest.raises(NotImplementedError):
        Adam([p], amsgrad=True)
    q = torch.zeros(4, dtype=torch.float64, device=device, requires_grad=True)
    q.grad = torch.zeros_like(q)
    with pytest.raises(TypeError):
        Adam([q]).step()


def test_adam_state_dict_roundtrip(device):
    """A loaded state continues exactly like the optimizer it came from (the tables are rebuilt)."""
    gen = torch.Generator().manual_seed(9)
    mk = lambda: [torch.randn(s, generator=gen).to(device).requires_grad_(True) for s in ((64, 32), (17,))]  # noqa: E731
    a = mk()
    b = [t.detach().clone().requires_grad_(True) for t in a]
    oa = Adam(a, lr=1e-2)
    grads = [[torch.randn(t.shape, generator=gen).to(device) for t in a] for _ in range(3)]
    for g in grads[:2]:
        for t, gg in zip(a, g):
            t.grad = gg.clone()
        oa.step()
    ob = Adam(b, lr=1e-2)
    with torch.no_grad():
        for t, s in zip(b, a):
            t.copy_(s)
    ob.load_state_dict(copy.deepcopy(oa.state_dict()))  # load_state_dict keeps same-device tensors as they are
    for t, s, gg in zip(b, a, grads[2]):
        t.grad = gg.clone()
        s.grad = gg.clone()
    oa.step()
    ob.step()
    for t, s in zip(b, a):
        torch.testing.assert_close(t, s, rtol=0, atol=0)


def test_adam_bumps_versions(device):
    """The kernel updates parameters in place: their version counters move as with an in-place torch op
    (version-keyed caches such as dense.weight_shadow's bf16 shadows rely on it)."""
    p = torch.ones(10, device=device, requires_grad=True)
    p.grad = torch.ones_like(p)
    v0 = p._version
    Adam([p], lr=0.1).step()
    assert p._version > v0 and float(p.detach()[0]) < 1.0


def test_adam_skips_params_without_grad(device):
    """parameters whose .grad is None are skipped as torch.optim.Adam skips them (their
    state stays empty / at its step), and a parameter that gets a gradient later starts its own step
    count; against torch.optim.Adam over 4 steps with a changing subset of gradients."""
    gen = torch.Generator().manual_seed(11)
    shapes = [(64, 33), (17,), (5, 5), (4097,)]
    ref = [torch.randn(s, generator=gen).to(device).requires_grad_(True) for s in shapes]
    got = [r.detach().clone().requires_grad_(True) for r in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-2, weight_decay=0.01)
    o_got = Adam(got, lr=1e-2, weight_decay=0.01)
    subsets = [(0, 1), (0, 1), (0, 1, 2, 3), (1, 3)]
    for sub in subsets:
        for i, (a, b) in enumerate(zip(ref, got)):
            if i in sub:
                g = torch.randn(a.shape, generator=gen).to(device)
                a.grad, b.grad = g.clone(), g.clone()
            else:
                a.grad = b.grad = None
        o_ref.step()
        o_got.step()
    for a, b in zip(ref, got):
        torch.testing.assert_close(b, a, rtol=2e-6, atol=1e-7)
        assert int(o_got.state[b]["step"]) == int(o_ref.state[a]["step"])
