"""Parity of the HIP edge-softmax + aggregation kernels against the CPU oracle (GPU).

Tolerance (fp32 kernel vs fp64 oracle):
    |got - ref| <= 1e-5 + 1e-4 * |ref|        per output and per gradient element
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle.pyg_gatv2 import gatv2_segment_reference

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-5, 1e-4


def close(got, ref, atol=ATOL, rtol=RTOL, msg=""):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else got
    ref = ref.detach().double().cpu().numpy() if torch.is_tensor(ref) else ref
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=atol, err_msg=msg)


def oracle_attention(XL, XR, att, bias, dst, N, gout, src=None):
    """fp64 oracle fwd + autograd bwd on the same inputs."""
    XLd = XL.detach().double().cpu().requires_grad_(True)
    XRd = XR.detach().double().cpu().requires_grad_(True)
    attd = att.detach().double().cpu().requires_grad_(True)
    biasd = bias.detach().double().cpu().requires_grad_(True)
    H, C = attd.shape
    XLe = XLd if src is None else XLd.index_select(0, src.cpu())
    out, smax, ssum = gatv2_segment_reference(XLe.view(-1, H, C), XRd.view(-1, H, C), attd, biasd, dst.cpu(), N)
    (out * gout.double().cpu()).sum().backward()
    return out, smax, ssum, XLd.grad, XRd.grad, attd.grad, biasd.grad


def random_graph(rng, N, E, empty_frac=0.1, sorted_dst=False):
    # destination distribution with some empty segments and a few heavy ones
    w = rng.random(N) ** 3
    w[rng.random(N) < empty_frac] = 0
    if w.sum() == 0:
        w[0] = 1
    dst = rng.choice(N, size=E, p=w / w.sum())
    if sorted_dst:
        dst = np.sort(dst)
    return torch.from_numpy(dst.astype(np.int64))


SHAPES = [(4, 1), (4, 8), (4, 16), (4, 256), (1, 32), (1, 64), (4, 32), (4, 64), (3, 5), (2, 3)]


@pytest.mark.parametrize("H,C", SHAPES)
@pytest.mark.parametrize("sorted_dst", [False, True])
@pytest.mark.parametrize("max_piece", [256, 7])
def test_attention_fwd_bwd_random(device, H, C, sorted_dst, max_piece):
    from gasfm_amd.attention import AttnPlan, GatAttentionFn
    rng = np.random.default_rng(H * 1000 + C + 7 * sorted_dst + max_piece)
    HC = H * C
    N, E = (50, 3000) if HC <= 64 else (6, 400)
    dst = random_graph(rng, N, E, sorted_dst=sorted_dst)
    plan = AttnPlan.from_targets(dst, N, max_piece=max_piece).to(device)
    XL = torch.randn(E, HC, device=device)
    XR = torch.randn(N, HC, device=device)
    att = torch.randn(H, C, device=device) * (1.0 / C ** 0.5)
    bias = torch.randn(HC, device=device)
    XL.requires_grad_(True)
    XR.requires_grad_(True)
    att.requires_grad_(True)
    bias.requires_grad_(True)
    out, smax, ssum = GatAttentionFn.apply(XL, XR, att, bias, plan, H, 0.2)
    gout = torch.randn(N, HC, device=device)
    (out * gout).sum().backward()
    r_out, r_max, r_sum, r_dXL, r_dXR, r_datt, r_dbias = oracle_attention(XL, XR, att, bias, dst, N, gout)
    close(out, r_out, msg="out")
    nonempty = torch.bincount(dst, minlength=N) > 0
    close(smax[nonempty.to(device)], r_max[nonempty], msg="seg_max")
    close(ssum, r_sum, msg="seg_sum")
    close(XL.grad, r_dXL, msg="dXL")
    close(XR.grad, r_dXR, msg="dXR")
    close(att.grad, r_datt, atol=1e-4, msg="datt")
    close(bias.grad, r_dbias, atol=1e-4, msg="dbias")


def test_empty_segments_give_bias_and_zero_grads(device):
    from gasfm_amd.attention import AttnPlan, GatAttentionFn
    N, H, C = 10, 4, 8
    dst = torch.tensor([2, 2, 5], dtype=torch.int64)
    plan = AttnPlan.from_targets(dst, N).to(device)
    XL = torch.randn(3, H * C, device=device, requires_grad=True)
    XR = torch.randn(N, H * C, device=device, requires_grad=True)
    att = torch.randn(H, C, device=device)
    bias = torch.randn(H * C, device=device)
    out, smax, ssum = GatAttentionFn.apply(XL, XR, att, bias, plan, H, 0.2)
    empty = [i for i in range(N) if i not in (2, 5)]
    close(out[empty], bias.expand(len(empty), -1), atol=0, rtol=0)
    assert torch.isfinite(out).all()
    out.sum().backward()
    assert torch.isfinite(XR.grad).all() and torch.isfinite(XL.grad).all()
    assert float(XR.grad[empty].abs().max()) == 0.0
    # single-edge segment: alpha == 1 -> out = XL + bias
    close(out[5], XL[2] + bias)


def test_dominant_logit_and_extreme_range(device):
    """Forces the online-max rescale: one huge logit inside a long split segment."""
    from gasfm_amd.attention import AttnPlan, GatAttentionFn
    H, C, E = 4, 8, 5000
    dst = torch.zeros(E, dtype=torch.int64)
    plan = AttnPlan.from_targets(dst, 1, max_piece=100).to(device)
    XL = torch.randn(E, H * C, device=device) * 0.1
    XL[3777] = 30.0  # far past every other logit, in a late piece
    XL[10] = -30.0
    XR = torch.randn(1, H * C, device=device)
    att = torch.ones(H, C, device=device)
    bias = torch.zeros(H * C, device=device)
    XL.requires_grad_(True)
    out, _, _ = GatAttentionFn.apply(XL, XR, att, bias, plan, H, 0.2)
    g = torch.randn(1, H * C, device=device)
    (out * g).sum().backward()
    r = oracle_attention(XL, XR, att, bias, dst, 1, g)
    close(out, r[0])
    close(XL.grad, r[3])


def test_permutation_invariance_within_segment(device):
    from gasfm_amd.attention import AttnPlan, gat_attention
    rng = np.random.default_rng(3)
    N, E, H, C = 40, 2000, 4, 8
    dst = random_graph(rng, N, E)
    XL = torch.randn(E, H * C, device=device)
    XR = torch.randn(N, H * C, device=device)
    att = torch.randn(H, C, device=device)
    bias = torch.randn(H * C, device=device)
    out1 = gat_attention(XL, XR, att, bias, AttnPlan.from_targets(dst, N).to(device), H)
    p = torch.from_numpy(rng.permutation(E))
    out2 = gat_attention(XL[p.to(device)], XR, att, bias, AttnPlan.from_targets(dst[p], N).to(device), H)
    close(out1, out2, atol=2e-6, rtol=1e-5)


def test_deterministic(device):
    from gasfm_amd.attention import AttnPlan, GatAttentionFn
    rng = np.random.default_rng(4)
    N, E, H, C = 100, 20000, 4, 8
    dst = random_graph(rng, N, E)
    plan = AttnPlan.from_targets(dst, N, max_piece=64).to(device)
    XL = torch.randn(E, H * C, device=device, requires_grad=True)
    XR = torch.randn(N, H * C, device=device, requires_grad=True)
    att = torch.randn(H, C, device=device, requires_grad=True)
    bias = torch.randn(H * C, device=device, requires_grad=True)
    res = []
    for _ in range(2):
        for t in (XL, XR, att, bias):
            t.grad = None
        out, _, _ = GatAttentionFn.apply(XL, XR, att, bias, plan, H, 0.2)
        out.square().sum().backward()
        res.append([out.detach().clone(), XL.grad.clone(), XR.grad.clone(), att.grad.clone()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _load_conv(f, device):
    from gasfm_amd.gatv2 import GATv2Conv
    H, C = f["att"].shape[1:]
    F_in = f["x"].shape[1]
    conv = GATv2Conv(F_in, C, heads=H, add_self_loops=False)
    with torch.no_grad():
        if "lin_l_w" in f.files:
            conv.lin_l.weight.copy_(torch.from_numpy(f["lin_l_w"]))
            conv.lin_r.weight.copy_(torch.from_numpy(f["lin_r_w"]))
        else:
            from oracle.weights import tensor_for
            key = str(f["weights_key"])
            conv.lin_l.weight.copy_(torch.from_numpy(tensor_for(key + ".lin_l.weight", (H * C, F_in))))
            conv.lin_r.weight.copy_(torch.from_numpy(tensor_for(key + ".lin_r.weight", (H * C, F_in))))
        conv.lin_l.bias.copy_(torch.from_numpy(f["lin_l_b"]))
        conv.lin_r.bias.copy_(torch.from_numpy(f["lin_r_b"]))
        conv.att.copy_(torch.from_numpy(f["att"]))
        conv.bias.copy_(torch.from_numpy(f["bias"]))
    return conv.to(device)


@pytest.mark.parametrize("name", ["conv_2_4_1_p2s.npz", "conv_2_4_1_p2v.npz", "conv_32_4_8_p2s.npz",
                                  "conv_32_4_8_p2v.npz", "conv_64_4_16_s2g.npz", "conv_1024_4_256_v2g.npz"])
def test_pyg_call_form_matches_reference_fixture(device, name):
    """gasfm_amd.GATv2Conv as a drop-in for torch_geometric.nn.GATv2Conv inside the reference's wrapper calls."""
    f = golden(name)
    conv = _load_conv(f, device)
    x = torch.from_numpy(f["x"]).float().to(device).requires_grad_(True)
    N = int(f["num_targets"])
    out = conv(x, torch.from_numpy(f["edge_index"]).to(device))[-N:]
    close(out, f["out"])
    (out * torch.from_numpy(f["gout"]).float().to(device)).sum().backward()
    close(x.grad, f["dx"], atol=2e-5)
    close(conv.att.grad, f["d_att"], atol=1e-4)
    close(conv.bias.grad, f["d_bias"], atol=1e-4)
    close(conv.lin_l.bias.grad, f["d_lin_l_b"], atol=1e-4)
    close(conv.lin_r.bias.grad, f["d_lin_r_b"], atol=1e-4)
    if "d_lin_l_w" in f.files:
        close(conv.lin_l.weight.grad, f["d_lin_l_w"], atol=1e-4)
        close(conv.lin_r.weight.grad, f["d_lin_r_w"], atol=1e-4)
    else:
        r = torch.from_numpy(f["r"]).float().to(device)
        close(conv.lin_l.weight.grad @ r, f["d_lin_l_w_r"], atol=1e-3, rtol=1e-3)
        close(conv.lin_r.weight.grad @ r, f["d_lin_r_w_r"], atol=1e-3, rtol=1e-3)


def test_pyg_call_form_repeated_sources(device):
    """General graph (a source with several out-edges): gathered path."""
    from gasfm_amd.gatv2 import GATv2Conv
    torch.manual_seed(0)
    conv = GATv2Conv(16, 8, heads=4, add_self_loops=False).to(device)
    x = torch.randn(30, 16, device=device, requires_grad=True)
    src = torch.randint(0, 30, (200,))
    dst = torch.randint(0, 30, (200,))
    out = conv(x, torch.stack([src, dst]).to(device))
    g = torch.randn_like(out)
    (out * g).sum().backward()
    xd = x.detach().double().cpu().requires_grad_(True)
    XL = (xd @ conv.lin_l.weight.double().cpu().T + conv.lin_l.bias.double().cpu())
    XR = (xd @ conv.lin_r.weight.double().cpu().T + conv.lin_r.bias.double().cpu())
    r_out, *_ = gatv2_segment_reference(XL[src].view(-1, 4, 8), XR.view(-1, 4, 8),
                                        conv.att.detach().double().cpu().view(4, 8),
                                        conv.bias.detach().double().cpu(), dst, 30)
    close(out, r_out)
    (r_out * g.double().cpu()).sum().backward()
    close(x.grad, xd.grad, atol=2e-5)


@pytest.mark.parametrize("H,C,E,max_piece", [(4, 16, 20000, 16), (4, 256, 1000, 8), (4, 8, 5000, 4)])
def test_single_target_two_level_combine(device, H, C, E, max_piece):
    """Global-style star (every source -> one target through a source permutation) split into
    hundreds of pieces: both combine levels in the forward and in the dXR backward sum."""
    from gasfm_amd.attention import AttnPlan, GatAttentionFn
    rng = np.random.default_rng(E + C)
    HC = H * C
    rows = E + 37
    src = torch.from_numpy(np.sort(rng.choice(rows, size=E, replace=False)).astype(np.int64))
    dst = torch.zeros(E, dtype=torch.int64)
    plan = AttnPlan.from_targets(dst, 1, src=src, src_rows=rows, max_piece=max_piece).to(device)
    assert plan.n_l1 > 1 and plan.n_part_rows == plan.n_slots + plan.n_l1
    XL = torch.randn(rows, HC, device=device, requires_grad=True)
    XR = torch.randn(1, HC, device=device, requires_grad=True)
    att = (torch.randn(H, C, device=device) / C ** 0.5).requires_grad_(True)
    bias = torch.randn(HC, device=device, requires_grad=True)
    out, smax, ssum = GatAttentionFn.apply(XL, XR, att, bias, plan, H, 0.2)
    gout = torch.randn(1, HC, device=device)
    (out * gout).sum().backward()
    r_out, r_max, r_sum, r_dXL, r_dXR, r_datt, r_dbias = oracle_attention(XL, XR, att, bias, dst, 1, gout, src=src)
    close(out, r_out, msg="out")
    close(smax, r_max, msg="seg_max")
    close(ssum, r_sum, rtol=2e-4, msg="seg_sum")
    close(XL.grad, r_dXL, msg="dXL")
    close(XR.grad, r_dXR, atol=1e-4, msg="dXR")
    close(att.grad, r_datt, atol=1e-4, msg="datt")
    close(bias.grad, r_dbias, atol=1e-4, msg="dbias")
