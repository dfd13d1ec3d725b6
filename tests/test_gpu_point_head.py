"""PointHeadFn (csrc/point_head.hip) against the scene-point head as the reference runs it
(code/models/graph_attn_sfm.py:170-174: pts3D = [scenepoint_head(relu(p))^T ; 1], the head
Linear(64,64) ReLU Linear(64,64) ReLU Linear(64,3), layers.py:10-44 norm=False).

Reference values: the same sequence in fp64.  Tolerance: the fused kernels sum in fp32 in a
different order than aten, so each result must lie within 10x the fp32 aten result's own
deviation from fp64 (plus 1e-6 of the output's scale) -- the principled bound used by the
training-step tests.  Row 3 must be exactly 1; repeated runs must be bit-identical.
"""
import pytest
import torch
import torch.nn.functional as F

from gasfm_amd import point_block
from gasfm_amd.model import get_linear_layers

pytestmark = pytest.mark.gpu


def _head(seed, device):
    torch.manual_seed(seed)
    return get_linear_layers(3 * [64] + [3], norm=False).to(device)


def _aten(seq, p):
    out = seq(F.relu(p)).T
    return torch.cat([out, torch.ones(1, out.shape[1], dtype=out.dtype, device=out.device)])


def _within(ours, aten, ref, what):
    dev = (aten.double() - ref).abs().max().item()
    err = (ours.double() - ref).abs().max().item()
    scale = ref.abs().max().item() if ref.numel() else 0.0
    assert err <= 10 * dev + 1e-6 * scale + 1e-12, f"{what}: err {err:.3e} vs aten fp32 {dev:.3e}"


@pytest.mark.parametrize("N", [1, 15, 16, 17, 1000, 40_013, 200_000])
def test_forward_backward(device, N):
    seq = _head(N, device)
    g = torch.Generator(device="cpu").manual_seed(N + 1)
    p = torch.randn(N, 64, generator=g).to(device)
    dout = torch.randn(4, N, generator=g).to(device)
    assert point_block.head_fusable(seq, p)

    def run(fn, s, x):
        x = x.clone().requires_grad_(True)
        for prm in s.parameters():
            prm.grad = None
        y = fn(s, x)
        y.backward(dout)
        return [y.detach(), x.grad] + [prm.grad.clone() for prm in s.parameters()]

    ours = run(point_block.head, seq, p)
    aten = run(_aten, seq, p)
    seq64 = _head(N, device).double()
    seq64.load_state_dict({k: v.double() for k, v in seq.state_dict().items()})
    ref = run(_aten, seq64, p.double())
    names = ["pts3D", "dp"] + [n for n, _ in seq.named_parameters()]
    for o, a, r, name in zip(ours, aten, ref, names):
        assert o.shape == r.shape, name
        _within(o, a, r, name)
    assert bool((ours[0][3] == 1).all())
    again = run(point_block.head, seq, p)
    for o, a, name in zip(ours, again, names):
        assert torch.equal(o, a), f"{name} not deterministic"


def test_empty(device):
    seq = _head(0, device)
    p = torch.zeros(0, 64, device=device, requires_grad=True)
    y = point_block.head(seq, p)
    assert y.shape == (4, 0)
    y.sum().backward()
    assert p.grad.shape == (0, 64)
    assert all(float(prm.grad.abs().sum()) == 0.0 for prm in seq.parameters())


def test_other_heads_not_fused(device):
    """Heads other than the 64-64-3 MLP (another hidden-layer count, a norm) keep the aten path."""
    p = torch.randn(50, 64, device=device)
    assert not point_block.head_fusable(get_linear_layers(2 * [64] + [3], norm=False).to(device), p)
    assert not point_block.head_fusable(get_linear_layers(3 * [64] + [3], norm=True).to(device), p)
    assert not point_block.head_fusable(_head(1, device), p.double())
