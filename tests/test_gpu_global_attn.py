"""The fused global GATv2 convs (csrc/global_attn.hip: view->global and points->global in one
launch each way, layers.py:550-556, 566-572) vs an fp64 torch GATv2 with one target.

Tolerances: outputs elementwise 2e-5 * max|ref| + 1e-6 (fp32 online softmax over up to ~10^5
sources); gradients normwise 1e-4.  Edge cases: one source, chunk boundaries (64 views / 2048
points per workgroup), sources that skip rows (dXL rows of non-sources stay 0), a rank without
sources (S = 0), the sharded partial row, determinism.
"""
import pytest
import torch
import torch.nn.functional as F

from gasfm_amd import _native
from gasfm_amd.attention import AttnPlan, GlobalPairFn

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_global_convs(monkeypatch):
    """The fused kernels are taken for shard-size point sets only (attention.GATT_MAX_SRC): on for
    every size in these tests."""
    from gasfm_amd import attention
    monkeypatch.setattr(attention, "GLOBAL_ATTN", True)
    monkeypatch.setattr(attention, "GATT_MAX_SRC", 1 << 62)

H = 4
SLOPE = 0.2


def _ref(XL, XR, att, bias, src):
    """fp64 single-target GATv2: returns (out [1, HC], max [H], sum [H])."""
    C = att.numel() // H
    x = XL[src].view(-1, H, C)
    e = (F.leaky_relu(x + XR.view(1, H, C), SLOPE) * att.view(1, H, C)).sum(-1)  # [S, H]
    if e.shape[0] == 0:
        return bias.view(1, -1).clone(), torch.full((H,), -float("inf"), dtype=e.dtype), torch.zeros(H, dtype=e.dtype)
    M = e.max(0).values
    w = torch.exp(e - M)
    S = w.sum(0)
    out = (w.unsqueeze(-1) * x).sum(0) / (S.unsqueeze(-1) + 1e-16)
    return out.reshape(1, -1) + bias.view(1, -1), M, S


def _case(gen, rows, S, C, subset):
    r = lambda *s, sc=1.0: torch.randn(*s, generator=gen, dtype=torch.float64) * sc  # noqa: E731
    HC = H * C
    if subset:
        src = torch.randperm(rows, generator=gen)[:S].sort().values
    else:
        src = torch.arange(S)
    return dict(XL=r(rows, HC), XR=r(1, HC, sc=0.5), att=r(1, H, C, sc=C ** -0.5), bias=r(HC, sc=0.1), src=src)


def _plan(src, rows, device):
    return AttnPlan.from_targets(torch.zeros(len(src), dtype=torch.int64), 1, src=src, src_rows=rows).to(device)


@pytest.mark.parametrize("nv,Sv,sub_v", [(1, 1, False), (64, 64, False), (125, 65, True), (1000, 993, True)])
@pytest.mark.parametrize("npt,Sp,sub_p", [(1, 1, False), (2048, 2048, False), (4100, 2049, True),
                                          (100000, 100000, False)])
def test_global_pair_matches_fp64(device, nv, Sv, sub_v, npt, Sp, sub_p):
    gen = torch.Generator().manual_seed(nv * 7 + npt + Sv + Sp)
    v, p = _case(gen, nv, Sv, 256, sub_v), _case(gen, npt, Sp, 16, sub_p)
    leaves64 = [t.clone().requires_grad_(True) for t in (v["XL"], v["XR"], v["att"], v["bias"], p["XL"], p["XR"],
                                                          p["att"], p["bias"])]
    ov, _, _ = _ref(*leaves64[:4], v["src"])
    op, _, _ = _ref(*leaves64[4:], p["src"])
    x64 = torch.cat([ov, op], 1)
    gx = torch.randn(x64.shape, generator=gen, dtype=torch.float64)
    x64.backward(gx)
    got = [t.detach().float().to(device).requires_grad_(True) for t in leaves64]
    pv, pp = _plan(v["src"], nv, device), _plan(p["src"], npt, device)
    x = GlobalPairFn.apply(*got[:4], *got[4:], pv, pp, H, SLOPE)
    assert x.grad_fn.fused, "fused global conv kernels not taken"
    torch.testing.assert_close(x.double().cpu(), x64.detach(), rtol=0, atol=2e-5 * x64.abs().max().item() + 1e-6)
    x.backward(gx.float().to(device))
    names = ("XLv", "XRv", "att_v", "bias_v", "XLp", "XRp", "att_p", "bias_p")
    # absolute floor per conv: with one source alpha = 1 and dXR, datt vanish analytically; fp32
    # leaves the cancellation of gout . XL against gout . (out - bias), a rounding of the size
    # eps32 |gout| |XL[src]| (measured 2.4e-5 for att_v at C = 256, where this floor is 1.2e-4)
    HCv = ov.shape[1]
    floor = [1e-5 + 2.0 ** -23 * gx[:, sl].norm().item() * d["XL"][d["src"]].norm().item()
             for sl, d in ((slice(0, HCv), v), (slice(HCv, None), p))]
    for k, (nm, a, r) in enumerate(zip(names, got, leaves64)):
        ga, gr = a.grad.double().cpu(), r.grad
        err = (ga - gr).norm().item()
        bound = 1e-4 * gr.norm().item() + floor[k // 4]
        assert err <= bound, f"{nm}: {err:.3e} vs |ref| {gr.norm().item():.3e} (bound {bound:.3e})"
    if sub_v:  # rows that are not sources get exactly zero
        mask = torch.ones(nv, dtype=torch.bool)
        mask[v["src"]] = False
        assert got[0].grad.cpu()[mask].abs().max().item() == 0.0
    # deterministic: bitwise the same forward and gradients on a second pass
    first = [a.grad.clone() for a in got]
    for a in got:
        a.grad = None
    x2 = GlobalPairFn.apply(*got[:4], *got[4:], pv, pp, H, SLOPE)
    assert torch.equal(x2, x)
    x2.backward(gx.float().to(device))
    for a, f in zip(got, first):
        assert torch.equal(a.grad, f)


@pytest.mark.parametrize("Sv,Sp", [(0, 5000), (70, 0), (0, 0), (200, 3000)])
def test_partial_rows_match_fp64(device, Sv, Sp):
    """Sharded forward: the packed partial row [acc | max | sum] of each conv (acc relative to the
    row's own max), including a rank without sources (acc 0, max -inf, sum 0)."""
    gen = torch.Generator().manual_seed(Sv + 3 * Sp + 1)
    v, p = _case(gen, max(Sv, 1) + 3, Sv, 256, True), _case(gen, max(Sp, 1), Sp, 16, False)
    parts, probs = [], []
    for d, rows in ((v, v["XL"].shape[0]), (p, p["XL"].shape[0])):
        HC = d["att"].numel()
        part = torch.full((HC + 2 * H,), 7.0, device=device)
        plan = _plan(d["src"], rows, device)
        probs.append(dict(XL=d["XL"].float().to(device), src=plan.perm, S=plan.num_edges,
                          XR=d["XR"].float().to(device), att=d["att"].float().to(device).reshape(-1),
                          bias=d["bias"].float().to(device), part=part))
        parts.append(part)
    _native.gatt_fwd(probs, SLOPE)
    torch.cuda.synchronize()
    for d, part in zip((v, p), parts):
        HC = d["att"].numel()
        out, M, S = _ref(d["XL"], d["XR"], d["att"], d["bias"], d["src"])
        got = part.double().cpu()
        if len(d["src"]) == 0:
            assert torch.equal(got[:HC], torch.zeros(HC, dtype=torch.float64))
            assert torch.all(got[HC:HC + H] == -float("inf")) and torch.all(got[HC + H:] == 0)
            continue
        torch.testing.assert_close(got[HC:HC + H], M, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(got[HC + H:], S, rtol=1e-4, atol=0)
        fin = got[:HC].view(H, -1) / got[HC + H:].view(H, 1) + d["bias"].view(H, -1)
        torch.testing.assert_close(fin.view(1, -1), out, rtol=0, atol=2e-5 * out.abs().max().item() + 1e-6)


def test_backward_without_sources(device):
    """S = 0 on both convs (a rank that owns no views and no points): zero dXR / datt, dbias = gout."""
    f = dict(dtype=torch.float32, device=device)
    probs, outs = [], []
    for C in (256, 16):
        HC = H * C
        o = dict(dXR=torch.full((HC,), 3.0, **f), datt=torch.full((2 * HC,), 3.0, **f))
        gout = torch.randn(HC, **f)
        probs.append(dict(XL=torch.empty((0, HC), **f), src=None, S=0, XR=torch.randn(HC, **f),
                          att=torch.randn(HC, **f), bias=torch.randn(HC, **f), out=torch.randn(HC, **f),
                          smax=torch.zeros(H, **f), ssum=torch.ones(H, **f), gout=gout, dXL=None, **o))
        outs.append((o, gout))
    _native.gatt_bwd(probs, SLOPE)
    torch.cuda.synchronize()
    for o, gout in outs:
        HC = gout.numel()
        assert torch.all(o["dXR"] == 0) and torch.all(o["datt"][:HC] == 0)
        assert torch.equal(o["datt"][HC:], gout)


def test_model_takes_fused_global_convs(device):
    """The learning conf's blocks run both global convs through the fused kernels."""
    import gasfm_amd
    from gasfm_amd import synthetic
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=2)).to(device)
    data = gasfm_amd.SceneData.from_synthetic(synthetic.scaled_config4(0.01, seed=3)).to(device)
    pred = net(data)
    seen, todo, fused = set(), [pred["Ps_norm"].grad_fn], []
    while todo:
        fn = todo.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        if type(fn).__name__ == "GlobalPairFnBackward":
            fused.append(fn.fused)
        todo.extend(f for f, _ in fn.next_functions)
    assert fused and all(fused), fused


@pytest.mark.parametrize("W", [1, 2, 8])
def test_merge_of_gathered_rows_matches_fp64(device, W):
    """Sharded forward end to end: W ranks' partial rows (sources split in W contiguous ranges, one
    rank empty when W = 8) packed as ShardedGlobalAttentionFn packs them, merged by one
    gasfm_gatt_merge launch == the fp64 conv over all sources."""
    from gasfm_amd.distributed import _pack_layout
    gen = torch.Generator().manual_seed(11 * W)
    v, p = _case(gen, 1000, 1000, 256, False), _case(gen, 30000, 30000, 16, False)
    Lv, Lp = 1024 + 2 * H, 64 + 2 * H
    B, ov = _pack_layout(Lv, Lp)
    g = torch.zeros(W * B, device=device)
    for r in range(W):
        probs = []
        for d, off, L in ((v, 0, Lv), (p, ov, Lp)):
            n = d["XL"].shape[0]
            bounds = [(n * k) // W for k in range(W + 1)]
            if W == 8:
                bounds[6] = bounds[5]  # rank 5 owns no sources (rank 6 takes its range)
            lo, hi = bounds[r], bounds[r + 1]
            XL = d["XL"][lo:hi].float().to(device)
            probs.append(dict(XL=XL if hi > lo else torch.empty((0, L - 2 * H), device=device), src=None, S=hi - lo,
                              XR=d["XR"].float().to(device), att=d["att"].float().to(device).reshape(-1),
                              bias=d["bias"].float().to(device), part=g[r * B + off:r * B + off + L]))
        _native.gatt_fwd(probs, SLOPE)
    xcat = torch.empty((1, 1024 + 64), device=device)
    stats = torch.empty((4, H), device=device)
    _native.gatt_merge([dict(part=g, bias=v["bias"].float().to(device), out=xcat[:, :1024], smax=stats[0],
                             ssum=stats[1]),
                        dict(part=g[ov:], bias=p["bias"].float().to(device), out=xcat[:, 1024:], smax=stats[2],
                             ssum=stats[3])], W, B)
    torch.cuda.synchronize()
    for d, o, k in ((v, xcat[:, :1024], 0), (p, xcat[:, 1024:], 2)):
        out, M, S = _ref(d["XL"], d["XR"], d["att"], d["bias"], torch.arange(d["XL"].shape[0]))
        torch.testing.assert_close(o.double().cpu(), out, rtol=0, atol=2e-5 * out.abs().max().item() + 1e-6)
        torch.testing.assert_close(stats[k].double().cpu(), M, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(stats[k + 1].double().cpu(), S, rtol=1e-4, atol=0)
