"""Single-row (global node) LayerNorm -> ReLU -> Linear (+ residual) kernels vs fp64 torch.

Shapes are the ones GASFM's global node uses (csrc/global_vec.hip header) plus the reduced
widths of the small test conf.  Tolerance: output elementwise 2e-5 * max|ref| + 1e-6;
gradients normwise 1e-4 (fp32 reductions over up to 2048 terms).
"""
import pytest
import torch
import torch.nn.functional as F

from gasfm_amd import dense

pytestmark = pytest.mark.gpu

SHAPES = [(2048, 1024), (2048, 64), (1024, 1024), (64, 64), (1088, 2048), (2048, 2048), (2048, 32), (128, 64),
          (192, 128)]


def _close(got, ref, name, tol=1e-4):
    err = (got.double().cpu() - ref).norm().item()
    assert err <= tol * ref.norm().item() + 1e-9, f"{name}: {err:.3e} vs |ref| {ref.norm().item():.3e}"


@pytest.mark.parametrize("K,N", SHAPES)
@pytest.mark.parametrize("mode", ["ln", "ln_resid", "plain", "plain_res"])
def test_gvec_matches_fp64(device, K, N, mode):
    if mode == "ln_resid" and K != N:
        pytest.skip("residual of the input needs N == K")
    g = torch.Generator().manual_seed(K * 3 + N)
    x = torch.randn(1, K, generator=g, dtype=torch.float64) * 1.5 + 0.3
    W = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
    b = torch.randn(N, generator=g, dtype=torch.float64)
    gam = 1 + 0.2 * torch.randn(K, generator=g, dtype=torch.float64)
    bet = 0.1 * torch.randn(K, generator=g, dtype=torch.float64)
    res = torch.randn(1, N, generator=g, dtype=torch.float64)
    dy = torch.randn(1, N, generator=g, dtype=torch.float64)
    use_ln = mode.startswith("ln")
    leaves64 = [t.clone().requires_grad_(True) for t in (x, W, b, gam, bet, res)]
    x6, W6, b6, g6, bt6, r6 = leaves64
    h = F.relu(F.layer_norm(x6, (K,), g6, bt6, 1e-5)) if use_ln else x6
    y64 = F.linear(h, W6, b6)
    if mode == "ln_resid":
        y64 = y64 + x6
    if mode == "plain_res":
        y64 = y64 + r6
    y64.backward(dy)
    leaves = [t.float().to(device).requires_grad_(True) for t in (x, W, b, gam, bet, res)]
    xd, Wd, bd, gd, btd, rd = leaves
    y = dense.GlobalLinearFn.apply(xd, gd if use_ln else None, btd if use_ln else None, Wd, bd,
                                   rd if mode == "plain_res" else None, 1e-5, mode == "ln_resid")
    y.backward(dy.float().to(device))
    scale = y64.abs().max().item()
    torch.testing.assert_close(y.double().cpu(), y64.detach(), rtol=0, atol=2e-5 * scale + 1e-6)
    names = ["x", "W", "b", "gamma", "beta", "res"]
    for nm, a, r in zip(names, leaves, leaves64):
        if r.grad is None:
            assert a.grad is None or a.grad.abs().max().item() == 0, nm
            continue
        _close(a.grad, r.grad, f"{mode} K={K} N={N} d{nm}")


def test_gvec_dispatch_and_determinism(device):
    ln = torch.nn.LayerNorm(2048).to(device)
    lin = torch.nn.Linear(2048, 2048).to(device)
    x = torch.randn(1, 2048, device=device, requires_grad=True)
    outs = []
    for _ in range(2):
        x.grad = None
        lin.zero_grad()
        y = dense.ln_relu_linear(x, ln, lin, residual=True)
        assert type(y.grad_fn).__name__ == "GlobalLinearFnBackward"
        y.square().sum().backward()
        outs.append((y.detach().clone(), x.grad.clone(), lin.weight.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    torch.testing.assert_close(outs[0][0], x + lin(F.relu(ln(x))), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("G,V,S", [(2048, 1024, 64), (128, 64, 64)])
@pytest.mark.parametrize("with_skip", [True, False])
def test_global_hub_matches_fp64(device, G, V, S, with_skip):
    """GlobalHubFn (batched gvec launches) vs the fp64 composition of its four consumers."""
    from gasfm_amd.dense import GlobalHubFn
    gen = torch.Generator().manual_seed(G + V + with_skip)
    r = lambda *s, sc=1.0, sh=0.0: torch.randn(*s, generator=gen, dtype=torch.float64) * sc + sh  # noqa: E731
    ins = [r(1, G, sc=2, sh=0.1), r(G, sc=0.3, sh=1), r(G, sc=0.2), r(32, G, sc=G ** -0.5),
           r(G, sc=0.3, sh=1), r(G, sc=0.2), r(V, G, sc=G ** -0.5), r(V, sc=0.1),
           r(G, sc=0.3, sh=1), r(G, sc=0.2), r(S, G, sc=G ** -0.5), r(S, sc=0.1),
           r(V, V, sc=V ** -0.5), r(V, sc=0.1), r(S, S, sc=S ** -0.5), r(S, sc=0.1)]
    grads = [r(1, G) if with_skip else None, r(1, 32), r(1, V), r(1, S)]
    ref = [t.clone().requires_grad_(True) for t in ins]
    g, gA, bA, WA, gB, bB, WB, bWB, gC, bC, WC, bWC, WD, bD, WE, bE = ref
    ln = lambda x, w, b: F.relu(F.layer_norm(x, (G,), w, b, 1e-5))  # noqa: E731
    outs64 = (g, F.linear(ln(g, gA, bA), WA), F.linear(F.linear(ln(g, gB, bB), WB, bWB), WD, bD),
              F.linear(F.linear(ln(g, gC, bC), WC, bWC), WE, bE))
    torch.autograd.backward([o for o, d in zip(outs64, grads) if d is not None], [d for d in grads if d is not None])
    got = [t.float().to(device).requires_grad_(True) for t in ins]
    outs = GlobalHubFn.apply(*got, 1e-5)
    for name, o, r64 in zip(("skip", "SG", "XRv", "XRp"), outs, outs64):
        torch.testing.assert_close(o.double().cpu(), r64.detach(), rtol=0, atol=2e-5 * r64.abs().max().item() + 1e-5,
                                   msg=name)
    torch.autograd.backward([o for o, d in zip(outs, grads) if d is not None],
                            [d.float().to(device) for d in grads if d is not None])
    names = ("g", "gA", "bA", "WA", "gB", "bB", "WB", "bWB", "gC", "bC", "WC", "bWC", "WD", "bD", "WE", "bE")
    for name, a, r64 in zip(names, got, ref):
        ga, gr = a.grad.double().cpu(), r64.grad
        err = (ga - gr).norm().item()
        assert err <= 1e-4 * gr.norm().item() + 1e-6, f"{name}: {err:.3e} vs |ref| {gr.norm().item():.3e}"


@pytest.mark.parametrize("G,Kc,V,S", [(2048, 1088, 1024, 64), (128, 128, 64, 64)])
@pytest.mark.parametrize("hub", [True, False], ids=["hub", "last_block"])
@pytest.mark.parametrize("with_prev", [True, False], ids=["prev", "no_prev"])
@pytest.mark.parametrize("rows", [1, 5], ids=["row", "rows5"])
def test_global_chain_matches_fp64(device, G, Kc, V, S, hub, with_prev, rows):
    """GlobalChainFn (csrc/global_chain.hip: the block's global tail + every consumer of g, four
    launches each way) vs the fp64 composition of layers.py:527-603 and its consumers (:497-520,
    :928-935, the next convs' lin_r), on one row or on 5 (a 4-scene union batch + its pad scene:
    one global node per scene, the parameter gradients summed over them).  Tolerances as the gvec
    tests: outputs 2e-5 * max|ref|, gradients normwise 1e-4."""
    gen = torch.Generator().manual_seed(G + Kc + 2 * hub + with_prev + 7 * rows)
    r = lambda *s, sc=1.0, sh=0.0: torch.randn(*s, generator=gen, dtype=torch.float64) * sc + sh  # noqa: E731
    names = ["xcat", "prev", "W1", "b1", "gM", "bM", "W2", "b2", "gA", "bA", "WA",
             "gB", "bB", "WB", "bWB", "gC", "bC", "WC", "bWC", "WD", "bD", "WE", "bE"]
    vals = [r(rows, Kc, sc=1.5, sh=0.1), r(rows, G, sc=2), r(G, Kc, sc=Kc ** -0.5), r(G, sc=0.1), r(G, sc=0.3, sh=1),
            r(G, sc=0.2), r(G, G, sc=G ** -0.5), r(G, sc=0.1), r(G, sc=0.3, sh=1), r(G, sc=0.2), r(32, G, sc=G ** -0.5),
            r(G, sc=0.3, sh=1), r(G, sc=0.2), r(V, G, sc=G ** -0.5), r(V, sc=0.1),
            r(G, sc=0.3, sh=1), r(G, sc=0.2), r(S, G, sc=G ** -0.5), r(S, sc=0.1),
            r(V, V, sc=V ** -0.5), r(V, sc=0.1), r(S, S, sc=S ** -0.5), r(S, sc=0.1)]
    present = {k: (with_prev or k != "prev") and (hub or k in names[:11]) for k in names}
    ref = {k: v.clone().requires_grad_(True) for k, v in zip(names, vals) if present[k]}
    ln = lambda x, w, b: F.relu(F.layer_norm(x, (G,), w, b, 1e-5))  # noqa: E731
    x1 = F.linear(ref["xcat"], ref["W1"], ref["b1"]) + (ref["prev"] if with_prev else 0)
    g = x1 + F.linear(ln(x1, ref["gM"], ref["bM"]), ref["W2"], ref["b2"])
    outs64 = [g, F.linear(ln(g, ref["gA"], ref["bA"]), ref["WA"])]
    if hub:
        outs64 += [F.linear(F.linear(ln(g, ref["gB"], ref["bB"]), ref["WB"], ref["bWB"]), ref["WD"], ref["bD"]),
                   F.linear(F.linear(ln(g, ref["gC"], ref["bC"]), ref["WC"], ref["bWC"]), ref["WE"], ref["bE"])]
    douts = [r(*o.shape) for o in outs64]
    torch.autograd.backward(outs64, douts)
    got = {k: v.detach().float().to(device).requires_grad_(True) for k, v in ref.items()}
    ws = [got.get(k) for k in names[2:]]
    outs = dense.GlobalChainFn.apply(got["xcat"], got.get("prev"), *ws, 1e-5, 1e-5, False)
    assert len(outs) == len(outs64)
    for name, o, r64 in zip(("g", "SG", "XRv", "XRp"), outs, outs64):
        torch.testing.assert_close(o.double().cpu(), r64.detach(), rtol=0, atol=2e-5 * r64.abs().max().item() + 1e-5,
                                   msg=name)
    torch.autograd.backward(list(outs), [d.float().to(device) for d in douts])
    for k, a in got.items():
        ga, gr = a.grad.double().cpu(), ref[k].grad
        err = (ga - gr).norm().item()
        assert err <= 1e-4 * gr.norm().item() + 1e-6, f"{k}: {err:.3e} vs |ref| {gr.norm().item():.3e}"
    # deterministic: a second backward gives bitwise the same gradients
    first = {k: a.grad.clone() for k, a in got.items()}
    for a in got.values():
        a.grad = None
    outs = dense.GlobalChainFn.apply(got["xcat"], got.get("prev"), *ws, 1e-5, 1e-5, False)
    torch.autograd.backward(list(outs), [d.float().to(device) for d in douts])
    for k, a in got.items():
        assert torch.equal(a.grad, first[k]), k


def test_model_uses_global_chain(device):
    """The learning conf's blocks run their global node through GlobalChainFn (hub blocks and the
    last block's lin_global-only chain)."""
    import gasfm_amd
    from gasfm_amd import synthetic
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3)).to(device)
    sc = synthetic.scaled_config4(0.01, seed=2)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    pred = net(data)
    seen, todo = set(), [pred["Ps_norm"].grad_fn]
    names = []
    while todo:
        fn = todo.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        names.append(type(fn).__name__)
        todo.extend(f for f, _ in fn.next_functions)
    assert names.count("GlobalChainFnBackward") == 3, names.count("GlobalChainFnBackward")
    assert "GlobalHubFnBackward" not in names
