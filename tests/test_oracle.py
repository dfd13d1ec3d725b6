"""Pin the CPU oracle against the reference-generated golden fixtures (no GPU).

The fixtures in tests/golden were produced by the reference's own model/graph
code (tests/golden/make_golden.py); these tests show the oracle restatement
reproduces them, so the oracle can stand in for the reference on the GPU box.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import gasfm_ref, scenes
from oracle.pyg_gatv2 import GATv2Conv, gatv2_segment_reference
from oracle.weights import deterministic_state_dict

CONV_FIXTURES = ["conv_2_4_1_p2s.npz", "conv_2_4_1_p2v.npz", "conv_32_4_8_p2s.npz", "conv_32_4_8_p2v.npz",
                 "conv_64_4_16_s2g.npz", "conv_1024_4_256_v2g.npz"]


def scene_graph():
    s = golden("scene_config1.npz")
    vals, g = scenes.graph_from_dense(s["M"], s["Ns"])
    return s, vals, g


def test_scene_graph_matches_reference_build():
    s, vals, g = scene_graph()
    np.testing.assert_array_equal(g.cam.numpy(), s["indices"][0])
    np.testing.assert_array_equal(g.pt.numpy(), s["indices"][1])
    np.testing.assert_array_equal(g.valid_views.numpy(), s["valid_views"])
    np.testing.assert_array_equal(g.valid_pts.numpy(), s["valid_pts"])
    # values: reference normalises in fp32, the oracle in fp64
    np.testing.assert_allclose(vals, s["values"], atol=2e-7)
    E = s["values"].shape[0]
    # edge_index layout of the reference wrappers (dataset_utils.py:531-535)
    np.testing.assert_array_equal(s["p2v_edge_index"][0], np.arange(E))
    np.testing.assert_array_equal(s["p2v_edge_index"][1], E + s["indices"][0])
    np.testing.assert_array_equal(s["p2s_edge_index"][1], E + s["indices"][1])


def load_conv(f):
    H, C = f["att"].shape[1:]
    F_in = f["x"].shape[1]
    conv = GATv2Conv(F_in, C, heads=H, add_self_loops=False).double()
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
    return conv


@pytest.mark.parametrize("name", CONV_FIXTURES)
def test_pyg_restatement_reproduces_fixture(name):
    f = golden(name)
    conv = load_conv(f)
    x = torch.from_numpy(f["x"]).requires_grad_(True)
    N = int(f["num_targets"])
    out = conv(x, torch.from_numpy(f["edge_index"]))[-N:]
    np.testing.assert_allclose(out.detach().numpy(), f["out"], rtol=1e-12, atol=1e-12)
    (out * torch.from_numpy(f["gout"])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), f["dx"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(conv.att.grad.numpy(), f["d_att"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(conv.bias.grad.numpy(), f["d_bias"], rtol=1e-10, atol=1e-12)


def test_segment_reference_matches_pyg_sequence():
    f = golden("conv_32_4_8_p2s.npz")
    conv = load_conv(f)
    x = torch.from_numpy(f["x"])
    ei = torch.from_numpy(f["edge_index"])
    N = int(f["num_targets"])
    E = ei.shape[1]
    H, C = 4, 8
    XL = conv.lin_l(x[:E]).view(E, H, C)
    XR = conv.lin_r(x[E:]).view(N, H, C)
    out, _, _ = gatv2_segment_reference(XL.detach(), XR.detach(), conv.att.detach().view(H, C),
                                        conv.bias.detach(), ei[1] - E, N)
    np.testing.assert_allclose(out.numpy(), f["out"], rtol=1e-12, atol=1e-12)


def test_identity_att_zero_is_reference_sparse_mean():
    """PyG-free known answer: att = 0 -> out = SparseMat.mean(XL) + bias (sparse_utils.py:414-419)."""
    f = golden("conv_identity_mean.npz")
    feats = torch.from_numpy(f["feats"])
    XL = (feats @ torch.from_numpy(f["lin_l_w"]).T + torch.from_numpy(f["lin_l_b"])).view(-1, 4, 8)
    idx = torch.from_numpy(f["indices"])
    att = torch.zeros(4, 8, dtype=torch.float64)
    bias = torch.from_numpy(f["bias"])
    n, m = f["pt_out"].shape[0], f["cam_out"].shape[0]
    pt_out, _, _ = gatv2_segment_reference(XL, torch.zeros(n, 4, 8, dtype=torch.float64), att, bias, idx[1], n)
    cam_out, _, _ = gatv2_segment_reference(XL, torch.zeros(m, 4, 8, dtype=torch.float64), att, bias, idx[0], m)
    np.testing.assert_allclose(pt_out.numpy(), f["pt_out"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(cam_out.numpy(), f["cam_out"], rtol=1e-12, atol=1e-12)


def test_functional_net_small_forward_and_grads():
    s, _, g = scene_graph()
    vals = torch.from_numpy(s["values"]).double()
    f = golden("net_small.npz")
    sd = {k[3:]: torch.from_numpy(f[k]).clone().requires_grad_(True) for k in f.files if k.startswith("sd/")}
    out = gasfm_ref.forward(sd, vals, g)
    np.testing.assert_allclose(out["Ps_norm"].detach().numpy(), f["Ps_norm"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(out["pts3D"].detach().numpy(), f["pts3D"], rtol=1e-10, atol=1e-12)
    loss = (out["Ps_norm"] * torch.from_numpy(f["cP"])).sum() + (out["pts3D"] * torch.from_numpy(f["cX"])).sum()
    loss.backward()
    for k, p in sd.items():
        ref = f["grad/" + k]
        got = torch.zeros_like(p) if p.grad is None else p.grad  # block-0 lin_r.weight: zero in the reference
        np.testing.assert_allclose(got.numpy(), ref, rtol=1e-8, atol=1e-11, err_msg=k)


@pytest.mark.parametrize("tag,layers", [("learning12", 12), ("optim9", 9)])
def test_functional_full_width_nets(tag, layers):
    import gasfm_amd
    s, _, g = scene_graph()
    vals = torch.from_numpy(s["values"]).double()
    f = golden(f"net_{tag}.npz")
    conf = gasfm_amd.learning_conf() if layers == 12 else gasfm_amd.optim_conf()
    sd = deterministic_state_dict(gasfm_amd.GraphAttnSfMNet(conf).state_dict(), torch.float64)
    with torch.no_grad():
        out = gasfm_ref.forward(sd, vals, g)
    np.testing.assert_allclose(out["Ps_norm"].numpy(), f["Ps_norm"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(out["pts3D"].numpy(), f["pts3D"], rtol=1e-10, atol=1e-12)


# ---------------------------------------------------------------- ESFMLoss (loss_functions.py:85-123)
def _esfm_case(f, i):
    margin, eq, vo, hinge, w, dloss = f["variants"][i]
    return float(margin), bool(eq), bool(vo), bool(hinge), float(w), float(dloss)


@pytest.mark.parametrize("i", range(5))
@pytest.mark.parametrize("form", ["dense", "edges"])
def test_esfm_loss_restatement_reproduces_reference(i, form):
    from oracle import esfm_loss
    f = golden("esfm_loss.npz")
    margin, eq, vo, hinge, w, dloss = _esfm_case(f, i)
    m, n = int(f["m"]), int(f["n"])
    Ps = torch.from_numpy(f["Ps"]).requires_grad_(True)
    X = torch.from_numpy(f["pts3D"]).requires_grad_(True)
    cam, pt = torch.from_numpy(f["cam"]), torch.from_numpy(f["pt"])
    vals = torch.from_numpy(f["values"]).double()
    if form == "dense":
        nM, valid = esfm_loss.dense_measurements(cam, pt, vals, m, n)
        loss = esfm_loss.esfm_loss(Ps, X, nM, valid, margin, hinge, w, eq, vo)
    else:
        loss = esfm_loss.esfm_loss_edges(Ps, X, cam, pt, vals, margin, hinge, w, eq, vo)
    (loss * dloss).backward()
    np.testing.assert_allclose(loss.item(), f[f"v{i}_loss"], rtol=1e-12)
    np.testing.assert_allclose(Ps.grad.numpy(), f[f"v{i}_dPs"], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(X.grad.numpy(), f[f"v{i}_dpts3D"], rtol=1e-10, atol=1e-13)


def test_esfm_sparse_values_are_norm_M_entries():
    """x.values (what the HIP loss reads) == the reference's dense norm_M at the valid entries."""
    f = golden("scene_config1.npz")
    M, Ns = torch.from_numpy(f["M"]).double(), torch.from_numpy(f["Ns"]).double()
    m = Ns.shape[0]
    h = torch.cat([M.reshape(m, 2, -1), torch.ones(m, 1, M.shape[1], dtype=torch.float64)], dim=1)
    nM = (Ns @ h)[:, :2, :]  # geo_utils.normalize_M
    idx = torch.from_numpy(f["indices"])
    np.testing.assert_allclose(nM[idx[0], :, idx[1]].numpy(), f["values"], rtol=1e-6, atol=1e-6)


def test_repro_oracle_matches_reference_core_errors():
    """oracle/repro.py == the reference's compute_core_errors (tests/golden/core_errors.npz)."""
    from oracle import repro
    f = golden("core_errors.npz")
    err, mean = repro.reprojection_errors(f["M"].astype(np.float64), f["Ns"].astype(np.float64),
                                          f["Ps_norm"].astype(np.float64), f["pts3D"].astype(np.float64))
    np.testing.assert_allclose(err[f["cam"], f["pt"]], f["edge_errors"], rtol=2e-5, atol=1e-3)
    assert np.isnan(err[~repro.valid_points(f["M"])]).all()
    np.testing.assert_allclose(mean, f["our_repro"], rtol=1e-5)


def test_rotational_homography_draws_match_reference():
    """rotational_homography draws torch's CPU RNG in the reference's order: with the fixture's seed
    the camera update y' = Ns^-1 R Ns y reproduces the reference's augmented cameras."""
    from gasfm_amd.scene_device import rotational_homography
    f = golden("scene_aug.npz")
    nv, _, tseed, inplane, tilt = f["params"]
    Ns = torch.from_numpy(f["Ns"])[:int(nv)]  # config 1: every Ns is the same K^-1
    torch.manual_seed(int(tseed))
    R = rotational_homography(int(nv), inplane, tilt)
    y = (torch.linalg.inv(Ns) @ R @ Ns) @ torch.from_numpy(f["s_y"])
    np.testing.assert_allclose(y.numpy(), f["a_y"], rtol=2e-5, atol=1e-6)  # host BLAS rounding varies by CPU


def _oracle_step(f, scenes_keys, layers, loss_conf):
    """oracle fp64 forward of each scene + ESFMLoss restatement, summed, one backward."""
    from oracle import esfm_loss
    import gasfm_amd
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=layers))
    sd = {k: v.clone().requires_grad_(True) for k, v in
          deterministic_state_dict(net.state_dict(), torch.float64).items()}
    del net
    total = torch.zeros((), dtype=torch.float64)
    losses = []
    for Mk, Nk in scenes_keys:
        vals, g = scenes.graph_from_dense(f[Mk], f[Nk], fp32_values=True)
        vals = torch.as_tensor(vals, dtype=torch.float64)
        r = gasfm_ref.forward(sd, vals, g, dtype=torch.float64)
        loss = esfm_loss.esfm_loss_edges(r["Ps_norm"], r["pts3D"], g.cam, g.pt, vals, *loss_conf)
        losses.append(float(loss.detach()))
        total = total + loss
    total.backward()
    return losses, {k: v.grad for k, v in sd.items()}


LOSS_CONF = (1e-4, True, 1.0, True, True)  # margin, hinge, hinge_w, equalize, valid_only


def _check_projected(grads, f):
    """normwise 1e-9 (fp64 vs fp64; the measurements normalised in fp32 on both sides)."""
    from conftest import fixture_grad, project_grad
    for k, g in grads.items():
        ref, _ = fixture_grad(f, k)
        got = project_grad(k, g if g is not None else torch.zeros(1))
        assert np.linalg.norm(got - ref) <= 1e-9 * np.linalg.norm(ref) + 1e-15, k


def test_oracle_training_step_matches_reference_config2():
    """Config 2 (optim conf, 9 blocks, full width, ESFMLoss): the oracle's gradients == the reference's."""
    f = golden("net_optim9_grads.npz")
    losses, grads = _oracle_step(f, [("M", "Ns")], 9, LOSS_CONF)
    np.testing.assert_allclose(losses[0], float(f["loss"][()]), rtol=1e-10)
    _check_projected(grads, f)


def test_oracle_training_step_matches_reference_config3():
    """Config 3 (learning conf, 12 blocks): batch of two scenes, summed ESFMLoss, one backward."""
    f = golden("train_step12.npz")
    losses, grads = _oracle_step(f, [("M0", "Ns0"), ("M1", "Ns1")], 12, LOSS_CONF)
    np.testing.assert_allclose(losses, [float(f["loss0"][()]), float(f["loss1"][()])], rtol=1e-10)
    _check_projected(grads, f)
