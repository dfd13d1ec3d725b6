"""Parity of the HIP ESFMLoss (gasfm_amd.loss, csrc/esfm_loss.hip) against the reference's own
outputs (tests/golden/esfm_loss.npz, made by code/loss_functions.py:69-123) and the oracle
restatement (oracle/esfm_loss.py, pinned to that fixture in tests/test_oracle.py).

Tolerance (fp32 kernel vs fp64 reference):
    loss:   |got - ref| <= 1e-5 |ref|
    grads:  ||got - ref|| <= 1e-4 ||ref|| per tensor (normwise), |got - ref| <= 1e-4 max|ref|
The gradients are unit vectors / #valid-depth per edge, so fp32 roundoff is ~1e-7 relative;
the bounds leave room for the classification of depths within fp32 roundoff of the margin,
which the chosen inputs keep away from.
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from conftest import golden
from gasfm_amd.loss import ESFMLoss
from oracle import esfm_loss as oracle_loss

pytestmark = pytest.mark.gpu


def loss_conf(margin=1e-4, equalize=True, valid_only=True, hinge=True, hinge_w=1.0):
    return gasfm_amd.Conf({"model": {"view_head": {"enabled": True}, "scenepoint_head": {"enabled": True}},
                           "loss": {"infinity_pts_margin": margin,
                                    "pts_grad_equalization_pre_perspective_divide": equalize,
                                    "normalize_grad_wrt_valid_projections_only": valid_only, "hinge_loss": hinge,
                                    "hinge_loss_weight": hinge_w}})


def close(got, ref, name, tol=1e-4):
    got = got.detach().double().cpu().numpy()
    ref = np.asarray(ref.detach().cpu().numpy() if torch.is_tensor(ref) else ref, dtype=np.float64)
    nr = np.linalg.norm(ref)
    assert np.linalg.norm(got - ref) <= tol * nr + 1e-12, f"{name}: normwise {np.linalg.norm(got - ref):.3e} / {nr:.3e}"
    assert np.abs(got - ref).max() <= tol * np.abs(ref).max() + 1e-12, f"{name}: max abs"


def run(data, Ps, X, conf, dloss=1.0):
    Ps = Ps.detach().float().clone().requires_grad_(True)
    X = X.detach().float().clone().requires_grad_(True)
    loss = ESFMLoss(conf)({"Ps_norm": Ps, "pts3D": X}, data)
    (loss * dloss).backward()
    return loss, Ps.grad, X.grad


@pytest.mark.parametrize("i", range(5))
def test_matches_reference_fixture(device, i):
    f = golden("esfm_loss.npz")
    margin, eq, vo, hinge, w, dloss = (float(v) for v in f["variants"][i])
    data = gasfm_amd.SceneData.from_sparse(f["cam"], f["pt"], f["values"], int(f["m"]), int(f["n"])).to(device)
    conf = loss_conf(margin, bool(eq), bool(vo), bool(hinge), w)
    loss, dP, dX = run(data, torch.from_numpy(f["Ps"]).to(device), torch.from_numpy(f["pts3D"]).to(device), conf,
                       dloss)
    np.testing.assert_allclose(loss.item(), f[f"v{i}_loss"], rtol=1e-5)
    close(dP, f[f"v{i}_dPs"], "dPs")
    close(dX, f[f"v{i}_dpts3D"], "dpts3D")


def predictions(m, n, seed, device):
    g = torch.Generator().manual_seed(seed)
    Ps = torch.zeros((m, 3, 4), dtype=torch.float64)
    Ps[:, :, :3] = torch.eye(3, dtype=torch.float64) + 0.1 * torch.randn((m, 3, 3), generator=g, dtype=torch.float64)
    Ps[:, :, 3] = 0.3 * torch.randn((m, 3), generator=g, dtype=torch.float64)
    X = torch.randn((3, n), generator=g, dtype=torch.float64)
    X[2] = 2.0 + 1.5 * torch.randn(n, generator=g, dtype=torch.float64)
    X = torch.cat([X, torch.ones((1, n), dtype=torch.float64)])
    # round the fp64 inputs to fp32 so both sides see the same numbers
    return Ps.float().double().to(device), X.float().double().to(device)


def oracle_run(Ps, X, cam, pt, vals, conf_t, dloss=1.0):
    margin, eq, vo, hinge, w = conf_t
    Ps, X = Ps.clone().requires_grad_(True), X.clone().requires_grad_(True)
    loss = oracle_loss.esfm_loss_edges(Ps, X, cam, pt, vals.double(), margin, hinge, w, eq, vo)
    (loss * dloss).backward()
    return loss, Ps.grad, X.grad


VARIANTS = [(1e-4, True, True, True, 1.0), (1e-4, True, False, True, 1.0), (0.5, False, False, True, 0.7),
            (0.5, True, True, False, 0.0)]


@pytest.mark.parametrize("conf_t", VARIANTS)
@pytest.mark.parametrize("scale,max_piece", [(0.02, None), (0.05, 64)])
def test_scaled_config4_vs_oracle(device, conf_t, scale, max_piece):
    """Long camera segments (one workgroup per camera walks ~4k edges) and ~20-edge points."""
    from gasfm_amd import synthetic
    sc = synthetic.scaled_config4(scale, seed=5)
    data = gasfm_amd.SceneData.from_synthetic(sc, max_piece=max_piece).to(device)
    Ps, X = predictions(sc.m, sc.n, 9, device)
    margin, eq, vo, hinge, w = conf_t
    loss, dP, dX = run(data, Ps, X, loss_conf(margin, eq, vo, hinge, w))
    cam, pt = data.x.indices[0], data.x.indices[1]
    rl, rP, rX = oracle_run(Ps, X, cam, pt, data.x.values, conf_t)
    np.testing.assert_allclose(loss.item(), rl.item(), rtol=1e-5)
    close(dP, rP, "dPs")
    close(dX, rX, "dpts3D")


def test_edge_cases(device):
    """Zero reprojection error (torch's norm backward gives 0 there, so does normalize), a depth
    below the margin, a point with no valid depth, an empty camera and an empty point."""
    cam = np.array([0, 0, 0, 2, 2], dtype=np.int64)
    pt = np.array([0, 1, 3, 0, 3], dtype=np.int64)
    vals = np.array([[0.0, 0.0], [0.1, -0.2], [0.3, 0.3], [0.5, 0.25], [-0.1, 0.0]], dtype=np.float32)
    m, n = 3, 4
    Ps = torch.zeros((m, 3, 4), dtype=torch.float64)
    Ps[:, :, :3] = torch.eye(3, dtype=torch.float64)
    Ps[2, 2, 3] = -1.5  # camera 2 sees point 3 behind it
    X = torch.tensor([[0.0, 1.0, 7.0, 0.5], [0.0, -1.0, 7.0, 0.5], [1.0, 2.0, 7.0, 1.0], [1.0, 1.0, 1.0, 1.0]],
                     dtype=torch.float64)
    data = gasfm_amd.SceneData.from_sparse(cam, pt, vals, m, n).to(device)
    for conf_t in VARIANTS:
        margin, eq, vo, hinge, w = conf_t
        loss, dP, dX = run(data, Ps.to(device), X.to(device), loss_conf(margin, eq, vo, hinge, w), dloss=0.75)
        rl, rP, rX = oracle_run(Ps, X, torch.from_numpy(cam), torch.from_numpy(pt), torch.from_numpy(vals), conf_t,
                                dloss=0.75)
        np.testing.assert_allclose(loss.item(), rl.item(), rtol=1e-6)
        np.testing.assert_allclose(dP.cpu().numpy(), rP.numpy(), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(dX.cpu().numpy(), rX.numpy(), rtol=1e-5, atol=1e-7)


def test_all_depths_invalid(device):
    """#valid-depth = 0: the reference divides by max(1, 0) (loss_functions.py:107)."""
    cam, pt = np.array([0, 1], dtype=np.int64), np.array([0, 0], dtype=np.int64)
    vals = np.zeros((2, 2), dtype=np.float32)
    Ps = torch.zeros((2, 3, 4), dtype=torch.float64)
    Ps[:, :, :3] = torch.eye(3, dtype=torch.float64)
    X = torch.tensor([[0.2], [0.1], [-2.0], [1.0]], dtype=torch.float64)
    data = gasfm_amd.SceneData.from_sparse(cam, pt, vals, 2, 1).to(device)
    conf_t = VARIANTS[0]
    loss, dP, dX = run(data, Ps.to(device), X.to(device), loss_conf(*conf_t))
    rl, rP, rX = oracle_run(Ps, X, torch.from_numpy(cam), torch.from_numpy(pt), torch.from_numpy(vals), conf_t)
    np.testing.assert_allclose(loss.item(), rl.item(), rtol=1e-6)
    np.testing.assert_allclose(dP.cpu().numpy(), rP.numpy(), rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(dX.cpu().numpy(), rX.numpy(), rtol=1e-6, atol=1e-8)


def test_deterministic(device):
    from gasfm_amd import synthetic
    sc = synthetic.scaled_config4(0.05, seed=6)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    Ps, X = predictions(sc.m, sc.n, 4, device)
    a = run(data, Ps, X, loss_conf())
    b = run(data, Ps, X, loss_conf())
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_config4_full_size_vs_edge_oracle(device):
    """BASELINE config 4 (m = 1000, n = 200k, ~4M edges) against the fp64 edge-list oracle."""
    from gasfm_amd import synthetic
    sc = synthetic.config4()
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    Ps, X = predictions(sc.m, sc.n, 2, device)
    loss, dP, dX = run(data, Ps, X, loss_conf())
    rl, rP, rX = oracle_run(Ps, X, data.x.indices[0], data.x.indices[1], data.x.values, VARIANTS[0])
    np.testing.assert_allclose(loss.item(), rl.item(), rtol=1e-5)
    close(dP, rP, "dPs")
    close(dX, rX, "dpts3D")


def test_network_and_loss_backward(device):
    """The training step's loss end: GraphAttnSfMNet outputs -> ESFMLoss -> parameter grads, vs the
    functional oracle net + oracle loss in fp64 (net_small fixture weights)."""
    from conftest import check_grad
    from oracle import gasfm_ref, scenes
    f = golden("net_small.npz")
    s = golden("scene_config1.npz")
    data = gasfm_amd.SceneData(torch.from_numpy(s["M"]), torch.from_numpy(s["Ns"]), None, "config1").to(device)
    sd64 = {k[3:]: torch.from_numpy(f[k]) for k in f.files if k.startswith("sd/")}
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.conf.small_conf(2))
    net.load_state_dict({k: v.float() for k, v in sd64.items()})
    net = net.to(device)
    loss = ESFMLoss(loss_conf())(net(data), data)
    loss.backward()
    idx = torch.from_numpy(s["indices"])
    g = scenes.graph_from_edges(idx[0].numpy(), idx[1].numpy(), s["Ns"].shape[0], s["M"].shape[1])
    sdp = {k: v.clone().requires_grad_(True) for k, v in sd64.items()}
    vals = torch.from_numpy(s["values"]).double()
    r = gasfm_ref.forward(sdp, vals, g)
    rl = oracle_loss.esfm_loss_edges(r["Ps_norm"], r["pts3D"], idx[0], idx[1], vals, 1e-4, True, 1.0, True, True)
    rl.backward()
    np.testing.assert_allclose(loss.item(), rl.item(), rtol=1e-4)
    for k, p in net.named_parameters():
        ref = sdp[k].grad
        check_grad(p.grad, (torch.zeros_like(sdp[k]) if ref is None else ref).numpy(), k)
