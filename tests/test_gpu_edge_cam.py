"""The edge prologue with the camera attention fused in (csrc/edge_cam.hip, edge_block.EdgeCamFn).

Checked against an fp64 torch restatement of what it replaces -- the block's LayerNorm + ReLU
(layers.py:232-234), both convs' lin_l, the camera-direction GATv2 attention (PyG semantics,
oracle/pyg_gatv2.py; Proj2View's call, layers.py:329-335) and, for the backward, the block output's
residual / lin_proj path that the prologue's backward folds in (layers.py:245-261) -- with non-zero
attention, on camera plans with complete and split (partial + combined) items, and with and
without the LayerNorm (the final update's raw features, graph_attn_sfm.py:141-148).
Tolerance (fp32 vs fp64): |d| <= 1e-5 + 1e-4 |ref| for XLp, the aggregates, dP and dXR; weight /
attention gradients (sums over every edge) within 1e-4 of their largest element.
With the LayerNorm and the residual, EdgeCamFn also returns the block's lin_proj gradient (dwp,
the folded edge-epilogue weight gradient PROJ_SCALE sum_e dP'[e]^T [relu(LN(P[e])) | P0[e]],
layers.py:945-956), checked like the other weight gradients.
The model-level checks run the 3-block net with and without the fusion (GASFM_EDGE_CAM) and
against the fp64 functional oracle, and the 4-block net with the edge epilogue's backward folded
into edge_cam_pbwd (edge_block.EPI_FOLD) against the unfolded one.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import gasfm_amd
from gasfm_amd import _native, model, synthetic
from gasfm_amd.attention import AttnPlan
from gasfm_amd.edge_block import PROJ_SCALE, EdgeCamFn
from oracle.pyg_gatv2 import gatv2_segment_reference

pytestmark = pytest.mark.gpu


def close(got, ref, atol=1e-5, rtol=1e-4, msg=""):
    torch.testing.assert_close(got.detach().double(), ref.detach().double().to(got.device), atol=atol, rtol=rtol,
                               msg=lambda m: f"{msg}: {m}")


def close_sum(got, ref, msg=""):
    got, ref = got.detach().double(), ref.detach().double().to(got.device)
    bound = 1e-4 * float(ref.abs().max()) + 1e-6
    err = float((got - ref).abs().max())
    assert err <= bound, f"{msg}: max |err| {err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("ln", [True, False])
@pytest.mark.parametrize("max_piece", [256, 7])
@pytest.mark.parametrize("res", [True, False])
def test_edge_cam_fn_vs_fp64(device, ln, max_piece, res):
    sc = synthetic.scaled_config4(0.02, seed=3)
    E, m, n = sc.num_edges, sc.m, sc.n
    cam = torch.from_numpy(sc.cam.astype(np.int64))
    pt = torch.from_numpy(sc.pt.astype(np.int64))
    pc = AttnPlan.from_targets(cam, m, max_piece=max_piece).to(device)
    pp = AttnPlan.from_targets(pt, n).to(device)
    assert pc.perm is None and pp.pos is not None
    g = torch.Generator(device=device).manual_seed(5)
    rnd = lambda *s, sc=1.0: (torch.randn(s, generator=g, device=device) * sc)
    P = rnd(E, 32)
    ln_w = (1 + 0.3 * rnd(32)) if ln else None
    ln_b = (0.2 * rnd(32)) if ln else None
    Wpt, Wc, Wp = rnd(32, 32, sc=0.2), rnd(32, 32, sc=0.2), rnd(32, 34, sc=0.2)
    bpt, bc = rnd(32, sc=0.1), rnd(32, sc=0.1)
    XR, att, bias = rnd(m, 32), rnd(1, 4, 8, sc=0.35), rnd(32, sc=0.1)
    dwp = ln and res
    P0 = rnd(E, 2)
    leaves = [t for t in (P, ln_w, ln_b, Wpt, bpt, Wc, bc, XR, att, bias, Wp if dwp else None) if t is not None]
    for t in leaves:
        t.requires_grad_(True)
    gXLp, gout, dres = rnd(E, 32), rnd(m, 32), (rnd(E, 32) if res else None)
    with _native.dispatch_record():
        XLp, out_c, token = EdgeCamFn.apply(P, ln_w, ln_b, Wpt, bpt, Wc, bc, Wp, 1e-5, pp.pos, XR, att, bias, pc, 4,
                                            0.2, None, None, P0 if dwp else None, dwp)
    outs, grads = [XLp, out_c], [gXLp, gout]
    if res:
        outs.append(token)
        grads.append(dres)
    torch.autograd.backward(outs, grads)
    got = {id(t): t.grad for t in leaves}

    d = lambda t: None if t is None else t.detach().double().requires_grad_(True)
    Pd, lwd, lbd, Wptd, bptd, Wcd, bcd, XRd, attd, biasd = (d(t) for t in (P, ln_w, ln_b, Wpt, bpt, Wc, bc, XR, att,
                                                                            bias))
    x = F.relu(F.layer_norm(Pd, (32,), lwd, lbd, 1e-5)) if ln else Pd
    xlp = x @ Wptd.T + bptd
    xlc = x @ Wcd.T + bcd
    out_r, _, _ = gatv2_segment_reference(xlc.view(-1, 4, 8), XRd.view(-1, 4, 8), attd.view(4, 8), biasd,
                                          cam.to(device), m)
    L = (xlp * gXLp.double()).sum() + (out_r * gout.double()).sum()
    Wpd = Wp.detach().double().requires_grad_(True)
    if res:  # the block output P + (Wp [P_hat | P0] + ...) / 4 as seen from this prologue
        L = L + (dres.double() * (Pd + PROJ_SCALE * (x @ Wpd[:, :32].T + P0.double() @ Wpd[:, 32:].T))).sum()
    L.backward()
    XLp_edge = XLp[pp.pos.long()]  # row pos[e] holds edge e
    close(XLp_edge, xlp, msg="XLp")
    close(out_c, out_r, msg="camera aggregates")
    close(got[id(P)], Pd.grad, msg="dP")
    close(got[id(XR)], XRd.grad, atol=1e-4, msg="dXR")
    for name, t, r in (("dWpt", Wpt, Wptd), ("dbpt", bpt, bptd), ("dWc", Wc, Wcd), ("dbc", bc, bcd),
                       ("datt", att, attd), ("dbias", bias, biasd)):
        close_sum(got[id(t)], r.grad, msg=name)
    if ln:
        close_sum(got[id(ln_w)], lwd.grad, msg="dgamma")
        close_sum(got[id(ln_b)], lbd.grad, msg="dbeta")
    if dwp:
        close_sum(got[id(Wp)], Wpd.grad, msg="dWp (folded epilogue)")


@pytest.mark.parametrize("fused", [True, False])
def test_three_block_net_fused_vs_oracle(device, fused):
    """The 3-block learning-conf net with the fused prologue + camera attention (the default) and
    without it, against the fp64 oracle: outputs and every parameter gradient."""
    from conftest import check_grad, oracle_grads
    from oracle.weights import deterministic_state_dict
    prev = model.EDGE_CAM
    model.EDGE_CAM = fused
    try:
        sc = synthetic.scaled_config4(0.05, seed=11)
        data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
        net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
        sd = deterministic_state_dict(net.state_dict(), torch.float64)
        net.load_state_dict({k: v.float() for k, v in sd.items()})
        net = net.to(device)
        gen = torch.Generator().manual_seed(3)
        cP = torch.randn((sc.m, 3, 4), generator=gen, dtype=torch.float64)
        cX = torch.randn((4, sc.n), generator=gen, dtype=torch.float64)
        with _native.dispatch_record() as rec:
            pred = net(data)
            ((pred["Ps_norm"] * cP.float().to(device)).sum() + (pred["pts3D"] * cX.float().to(device)).sum()).backward()
            torch.cuda.synchronize()
        # 32-wide streamed attention forwards (blocks 1, 2 and the final update): the point direction
        # only when fused, point + camera otherwise
        n32 = rec.counts["attn_fwd_glds"] + rec.counts["attn_fwd_grp"]
        assert n32 == (3 if fused else 6), rec.counts
        (g64, r64), (g32, _) = oracle_grads(sd, sc, cP, cX)
        np.testing.assert_allclose(pred["Ps_norm"].detach().cpu().numpy(), r64["Ps_norm"].detach().numpy(),
                                   atol=1e-4, rtol=1e-3)
        np.testing.assert_allclose(pred["pts3D"].detach().cpu().numpy(), r64["pts3D"].detach().numpy(),
                                   atol=1e-4, rtol=1e-3)
        for k, p in net.named_parameters():
            check_grad(p.grad, g64[k], k, g32[k])
    finally:
        model.EDGE_CAM = prev


def test_epilogue_fold_vs_unfolded(device, monkeypatch):
    """The 4-block net (three seams) with the edge epilogue's backward folded into edge_cam_pbwd
    against the same net with edge_epilogue_bwd: identical forward, no edge_epilogue_bwd launch left,
    the lin_proj gradients (now edge_cam_pbwd's) within 1e-4 normwise of the unfolded ones, and every
    parameter gradient within 1e-3 normwise of the unfolded one or within 10x the unfolded one's own
    distance from the fp64 oracle (the smallest gradients, blocks down, amplify the summation-order
    differences past 1e-3).  test_three_block_net_fused_vs_oracle checks the folded path (the default)
    against the fp64 oracle alone."""
    from conftest import oracle_grads
    from gasfm_amd import edge_block
    from oracle.weights import deterministic_state_dict
    sc = synthetic.scaled_config4(0.05, seed=11)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=4))
    sd = deterministic_state_dict(net.state_dict(), torch.float64)
    net.load_state_dict({k: v.float() for k, v in sd.items()})
    net = net.to(device)
    gen = torch.Generator().manual_seed(3)
    cP = torch.randn((sc.m, 3, 4), generator=gen, dtype=torch.float64)
    cX = torch.randn((4, sc.n), generator=gen, dtype=torch.float64)
    calls = []
    orig = _native.edge_epilogue_bwd
    monkeypatch.setattr(_native, "edge_epilogue_bwd", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    res = {}
    for fold in (False, True):
        monkeypatch.setattr(edge_block, "EPI_FOLD", fold)
        calls.clear()
        net.zero_grad(set_to_none=True)
        pred = net(data)
        ((pred["Ps_norm"] * cP.float().to(device)).sum() + (pred["pts3D"] * cX.float().to(device)).sum()).backward()
        torch.cuda.synchronize()
        res[fold] = (pred["Ps_norm"].detach().clone(), {k: p.grad.detach().double().cpu() for k, p in net.named_parameters()},
                     len(calls))
    assert torch.equal(res[True][0], res[False][0])
    assert res[False][2] == 3 and res[True][2] == 0, (res[False][2], res[True][2])
    (g64, _), _ = oracle_grads(sd, sc, cP, cX)
    for k, g0 in res[False][1].items():
        g1 = res[True][1][k]
        err = float((g1 - g0).norm())
        if k.endswith("lin_proj.weight") and "projection_feature_update" in k:
            assert err <= 1e-4 * float(g0.norm()) + 1e-9, (k, err, float(g0.norm()))
        own = float((g0 - torch.from_numpy(g64[k])).norm())
        assert err <= max(1e-3 * float(g0.norm()), 10 * own) + 1e-9, (k, err, own, float(g0.norm()))


def test_block0_seam_vs_separate(device, monkeypatch):
    """Block 0's epilogue run inside block 1's prologue + camera attention kernel (Seam0Fn,
    gasfm_edge0_seam_fwd) against the separate launches (EDGE_SEAM off: Block0EpilogueFn +
    EdgeCamFn, and the 32-wide epilogues unseamed as well): one block-0 seam launch, the same
    outputs within 1e-5, and every parameter gradient within 1e-3 normwise or within 10x the
    unseamed one's own distance from the fp64 oracle (as test_epilogue_fold_vs_unfolded)."""
    from conftest import oracle_grads
    from oracle.weights import deterministic_state_dict
    sc = synthetic.scaled_config4(0.05, seed=13)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
    sd = deterministic_state_dict(net.state_dict(), torch.float64)
    net.load_state_dict({k: v.float() for k, v in sd.items()})
    net = net.to(device)
    gen = torch.Generator().manual_seed(5)
    cP = torch.randn((sc.m, 3, 4), generator=gen, dtype=torch.float64)
    cX = torch.randn((4, sc.n), generator=gen, dtype=torch.float64)
    calls = []
    orig = _native.edge0_seam_fwd
    monkeypatch.setattr(_native, "edge0_seam_fwd", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    res = {}
    for seam in (False, True):
        monkeypatch.setattr(model, "EDGE_SEAM", seam)
        calls.clear()
        net.zero_grad(set_to_none=True)
        pred = net(data)
        ((pred["Ps_norm"] * cP.float().to(device)).sum() + (pred["pts3D"] * cX.float().to(device)).sum()).backward()
        torch.cuda.synchronize()
        res[seam] = (pred["Ps_norm"].detach().clone(), pred["pts3D"].detach().clone(),
                     {k: p.grad.detach().double().cpu() for k, p in net.named_parameters()}, len(calls))
    assert res[False][3] == 0 and res[True][3] == 1, (res[False][3], res[True][3])
    close(res[True][0], res[False][0], msg="Ps_norm")
    close(res[True][1], res[False][1], msg="pts3D")
    (g64, _), _ = oracle_grads(sd, sc, cP, cX)
    for k, g0 in res[False][2].items():
        err = float((res[True][2][k] - g0).norm())
        own = float((g0 - torch.from_numpy(g64[k])).norm())
        assert err <= max(1e-3 * float(g0.norm()), 10 * own) + 1e-9, (k, err, own, float(g0.norm()))
