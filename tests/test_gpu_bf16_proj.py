"""BASELINE config 5's "bf16 projections on MFMA": GraphAttnSfMNet with
set_projection_precision("bf16") against the fp64 oracle (reference code/models/ forward,
oracle/gasfm_ref.py).

What changes: the camera-side D x D products (Proj2View's MLP and graph_conv_view2global.lin_l,
layers.py:292-320, 352-358, 506-511; forward and both backward products) on the large-m GEMM path
(operands rounded to bf16, 2^-9 relative, fp32 accumulation; the small-m fused view chain stays
fp32: view_block._chain_ok), and the global node's chain (layers.py:497-533, 594-603, 928-935) on
bf16 weight shadows (round 5; fp32 accumulation, fp32 gradients).  Stated tolerance of this mode,
against the fp64 reference on the 12-block learning conf (scaled config 4):
    outputs    ||got - ref|| <= 2e-2 ||ref||        (Ps_norm, pts3D; normwise)
    gradient   ||G - G_ref|| <= 0.1 ||G_ref||       (all parameter gradients flattened into one
                                                     vector, as train.py:137 concatenates them)
    per tensor ||g - r|| <= 0.25 ||r|| + 1e-3 ||G_ref||
Measured at scale 0.02 / 12 blocks: outputs 2.3e-3 / 1.5e-4, whole gradient 4.4e-2, worst tensor
0.115 (block 0's proj2view lin_l bias, at the far end of 12 blocks of bf16 backward products).
The absolute term covers tensors whose gradient is ~1e-5 of the whole (the global-feature path's
lin_r / norm_and_proj_global2view): bf16 rounding of the large terms feeding them leaves them
with O(1) relative error but ~1e-7 of ||G_ref|| absolute.  Gradient errors of this size are
what bf16 mixed-precision training carries; test_bf16_training_tracks_fp32 checks the effect
that matters, an Adam trajectory of the config-2 shape (9-block optim conf, ESFMLoss).
The fp32 mode keeps its own 1e-3 / 1e-4 bounds (test_gpu_model.py); this test also checks that
the bf16 mode actually changed the numbers (the kernel ran) while staying inside the bounds.
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from oracle import gasfm_ref, scenes
from oracle.weights import deterministic_state_dict

pytestmark = pytest.mark.gpu

OUT_TOL, GRAD_TOL, PARAM_TOL, PARAM_ATOL = 2e-2, 0.1, 0.25, 1e-3


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("scale,layers,chain", [(0.02, 12, True), (0.05, 3, True), (0.05, 3, False)])
def test_bf16_projections_vs_oracle(device, scale, layers, chain, monkeypatch):
    """chain False: the view side through the bf16 GEMM kernel (the large-m path) at this small m."""
    from gasfm_amd import synthetic, view_block
    monkeypatch.setattr(view_block, "VIEW_CHAIN", chain)
    sc = synthetic.scaled_config4(scale, seed=11)
    vals = sc.normalized_values()
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=layers))
    sd = deterministic_state_dict(net.state_dict(), torch.float64)
    net.load_state_dict({k: v.float() for k, v in sd.items()})
    net = net.to(device)
    g = scenes.graph_from_edges(sc.cam, sc.pt, sc.m, sc.n)
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ref = gasfm_ref.forward(sdp, torch.from_numpy(vals).double(), g)
    gen = torch.Generator().manual_seed(3)
    cP = torch.randn(ref["Ps_norm"].shape, generator=gen, dtype=torch.float64)
    cX = torch.randn(ref["pts3D"].shape, generator=gen, dtype=torch.float64)
    ((ref["Ps_norm"] * cP).sum() + (ref["pts3D"] * cX).sum()).backward()

    res = {}
    for prec in ("fp32", "bf16"):
        net.set_projection_precision(prec)
        for p in net.parameters():
            p.grad = None
        pred = net(data)
        ((pred["Ps_norm"] * cP.float().to(device)).sum() + (pred["pts3D"] * cX.float().to(device)).sum()).backward()
        res[prec] = ({k: pred[k].detach().cpu().numpy() for k in ("Ps_norm", "pts3D")},
                     {k: p.grad.detach().cpu().numpy() for k, p in net.named_parameters()})
    out_err = {k: rel(res["bf16"][0][k], ref[k].detach().numpy()) for k in ("Ps_norm", "pts3D")}
    grad_err = {}
    for k in res["bf16"][1]:
        r = sdp[k].grad
        r = np.zeros(sdp[k].shape) if r is None else r.numpy()
        grad_err[k] = (np.linalg.norm(res["bf16"][1][k] - r), np.linalg.norm(r))
    g_err = np.sqrt(sum(e * e for e, _ in grad_err.values()))
    g_ref = np.sqrt(sum(n * n for _, n in grad_err.values()))
    worst = sorted(grad_err.items(), key=lambda kv: -kv[1][0] / (PARAM_TOL * kv[1][1] + PARAM_ATOL * g_ref))[:4]
    print(f"\nbf16 proj, scale {scale}, {layers} blocks: outputs rel {out_err}; whole gradient rel "
          f"{g_err / g_ref:.3e} (|G_ref| {g_ref:.3e}); tightest tensors "
          + "; ".join(f"{k} {e:.2e} vs |r| {n:.2e}" for k, (e, n) in worst))
    for k, e in out_err.items():
        assert e <= OUT_TOL, f"{k}: normwise {e:.3e} > {OUT_TOL}"
    assert g_err <= GRAD_TOL * g_ref, f"whole gradient: normwise {g_err:.3e} vs |G_ref| {g_ref:.3e}"
    for k, (e, n) in grad_err.items():
        assert e <= PARAM_TOL * n + PARAM_ATOL * g_ref, f"{k}: normwise {e:.3e} vs |ref| {n:.3e}"
    # the bf16 kernel ran: outputs moved off the fp32 result, by more than fp32 roundoff
    assert rel(res["bf16"][0]["Ps_norm"], res["fp32"][0]["Ps_norm"]) > 1e-6


def test_bf16_training_tracks_fp32(device):
    """30 Adam steps of single-scene optimisation (config 2 shape: optim_euc conf, 9 blocks, the
    40-view x 1500-point fixture scene, ESFMLoss) from the same init in fp32 and in bf16-projection
    mode: the bf16 loss stays within 5 % of the fp32 loss at every step (measured: within 0.4 %)
    and both descend."""
    from conftest import golden
    from gasfm_amd.loss import ESFMLoss
    f = golden("net_optim9_grads.npz")
    conf = gasfm_amd.optim_conf()
    conf.put("loss", {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
                      "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True,
                      "hinge_loss_weight": 1.0})
    data = gasfm_amd.SceneData(torch.from_numpy(np.asarray(f["M"], dtype=np.float32)),
                               torch.from_numpy(np.asarray(f["Ns"])), None, "optim").to(device)
    lossf = ESFMLoss(conf)
    traj = {}
    for prec in ("fp32", "bf16"):
        net = gasfm_amd.GraphAttnSfMNet(conf)
        net.load_state_dict(deterministic_state_dict(net.state_dict()))
        net = net.to(device).set_projection_precision(prec)
        opt = torch.optim.Adam(net.parameters(), lr=1e-4)
        losses = []
        for _ in range(30):
            opt.zero_grad()
            loss = lossf(net(data), data)
            loss.backward()
            opt.step()
            losses.append(float(loss.detach()))
        traj[prec] = np.array(losses)
    print("\nfp32", np.array2string(traj["fp32"][::5], precision=4), "\nbf16",
          np.array2string(traj["bf16"][::5], precision=4))
    assert np.all(np.isfinite(traj["bf16"]))
    assert np.all(np.abs(traj["bf16"] - traj["fp32"]) <= 0.05 * np.abs(traj["fp32"]))
    # the first Adam step from this init overshoots (0.049 -> 0.487, both modes); descent after it
    assert traj["fp32"][-1] < traj["fp32"][1] and traj["bf16"][-1] < traj["bf16"][1]


def test_gchain_bf16_shadows(device):
    """The global node's chain on bf16 weight shadows (dense.weight_shadow, set_projection_precision
    "bf16"): the shadows are the weights rounded to bf16, re-rounded by the next forward after an
    in-place weight update, and the chain's outputs move from the fp32 mode's by a bf16-sized amount
    (> 0: the shadows were read; <= 2e-2 normwise on the global features)."""
    from gasfm_amd import dense, synthetic
    sc = synthetic.scaled_config4(0.02, seed=5)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
    sd = deterministic_state_dict(net.state_dict(), torch.float64)
    net.load_state_dict({k: v.float() for k, v in sd.items()})
    net = net.to(device)
    with torch.no_grad():
        ref = net(data)["Ps_norm"].clone()
        net.set_projection_precision("bf16")
        dense._SHADOWS.clear()
        got = net(data)["Ps_norm"].clone()
    live = [(r(), sh) for r, sh, _, _ in dense._SHADOWS.values() if r() is not None]
    assert len(live) >= 7, len(live)  # W1, W2, WA and the hub's WB..WE of at least one block
    for w, sh in live:
        assert torch.equal(sh, w.detach().to(torch.bfloat16))
    d = rel(got.cpu().numpy(), ref.cpu().numpy())
    assert 0 < d <= 2e-2, d
    name, p = next((k, v) for k, v in net.named_parameters()
                   if k.endswith("view_and_scenepoint2global.mlp.0.weight"))
    with torch.no_grad():
        p.mul_(1.25)
        net(data)
    sh = next(s for r, s, _, _ in dense._SHADOWS.values() if r() is p)
    assert torch.equal(sh, p.detach().to(torch.bfloat16)), name
    net.refresh_weight_shadows()
    assert torch.equal(sh, p.detach().to(torch.bfloat16))
