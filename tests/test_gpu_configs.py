"""BASELINE configs 2 and 3 at their own scale, against the oracle / the reference's fixtures (GPU).

  config 2  single-scene optimisation step (optim_euc_gasfm.conf: 9 blocks, full widths) on the
            full-size synthetic stand-in for AlcatrazCourtyard (synthetic.config2_standin: 133
            views x 23,674 points, E = 142,104; the dataset is absent offline, so parity on the real
            scene is unpinned -- the shape is the one owed), model + ESFMLoss (its optim conf) +
            backward, against the fp64 oracle (oracle/gasfm_ref.py + oracle/esfm_loss.py, both pinned
            to the reference by tests/test_oracle.py).  The point direction runs the grouped forward
            (23,674 points -> 2,960 wave tasks), which the test asserts.
  config 3  the union-graph batch (gasfm_amd/batch.py: the batch as ONE forward) directly against
            train_step12.npz, the reference's own 12-block net + ESFMLoss + summed batch loss.

Tolerances as tests/test_gpu_train_step.py (fp32 vs fp64): loss 1e-4 relative (or 10x the fp32
oracle's own deviation), outputs 1e-4 + 1e-3 |ref|, gradients normwise 1e-3 (or 10x the fp32
oracle's error) with an absolute floor of 1e-6 x the step's largest per-tensor gradient norm.
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from conftest import check_fixture_grads, check_grad, golden, project_grad
from gasfm_amd import _native, synthetic
from gasfm_amd.loss import ESFMLoss
from oracle.weights import deterministic_state_dict

pytestmark = pytest.mark.gpu

LOSS = {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
        "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True, "hinge_loss_weight": 1.0}


def _conf(conf):
    conf.put("loss", dict(LOSS))
    return conf


def test_config2_standin_full_size_step_vs_oracle(device):
    from oracle import esfm_loss, gasfm_ref, scenes
    sc = synthetic.config2_standin()
    assert (sc.m, sc.n) == (133, 23674)
    conf = _conf(gasfm_amd.optim_conf())
    net = gasfm_amd.GraphAttnSfMNet(conf)
    sd64 = deterministic_state_dict(net.state_dict(), torch.float64)
    net.load_state_dict({k: v.float() for k, v in sd64.items()})
    net = net.to(device)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    with _native.dispatch_record() as rec:
        pred = net(data)
        loss = ESFMLoss(conf)(pred, data)
        loss.backward()
        torch.cuda.synchronize()
    assert rec.counts["attn_fwd_grp"] == 9, rec.counts  # blocks 1..8 + final update

    g = scenes.graph_from_edges(sc.cam, sc.pt, sc.m, sc.n)
    vals = torch.from_numpy(sc.normalized_values())
    refs = {}
    for dt in (torch.float64, torch.float32):
        sd = {k: v.to(dt).clone().requires_grad_(True) for k, v in sd64.items()}
        r = gasfm_ref.forward(sd, vals.to(dt), g, dtype=dt)
        lr = esfm_loss.esfm_loss_edges(r["Ps_norm"], r["pts3D"], g.cam, g.pt, vals.to(dt), 1e-4, True, 1.0, True, True)
        lr.backward()
        refs[dt] = (r, float(lr.detach()), {k: (v.grad if v.grad is not None else torch.zeros_like(v))
                                            for k, v in sd.items()})
    r64, l64, g64 = refs[torch.float64]
    _, l32, g32 = refs[torch.float32]
    np.testing.assert_allclose(pred["Ps_norm"].detach().cpu().numpy(), r64["Ps_norm"].detach().numpy(),
                               atol=1e-4, rtol=1e-3)
    np.testing.assert_allclose(pred["pts3D"].detach().cpu().numpy(), r64["pts3D"].detach().numpy(),
                               atol=1e-4, rtol=1e-3)
    rtol = max(1e-4, 10 * abs(l32 - l64) / abs(l64))
    np.testing.assert_allclose(float(loss.detach()), l64, rtol=rtol)
    p64 = {k: project_grad(k, v) for k, v in g64.items()}
    floor = 1e-6 * max(np.linalg.norm(v) for v in p64.values()) + 1e-9
    for k, p in net.named_parameters():
        check_grad(project_grad(k, p.grad), p64[k], k, project_grad(k, g32[k]), atol=floor)


def test_config3_union_batch_matches_reference_fixture(device):
    """forward_batch (one union-graph forward for the whole batch) vs train_step12.npz: per-scene
    losses, the summed batch loss and every parameter gradient, at test_gpu_train_step's bounds."""
    from gasfm_amd.batch import forward_batch
    f = golden("train_step12.npz")
    conf = _conf(gasfm_amd.learning_conf())
    net = gasfm_amd.GraphAttnSfMNet(conf)
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    net = net.to(device)
    lossf = ESFMLoss(conf)
    datas = [gasfm_amd.SceneData(torch.from_numpy(np.asarray(f[f"M{i}"], dtype=np.float32)),
                                 torch.from_numpy(np.asarray(f[f"Ns{i}"])), None, f"s{i}").to(device) for i in range(2)]
    preds = forward_batch(net, datas)
    losses = [lossf(p, d) for p, d in zip(preds, datas)]
    for i, l in enumerate(losses):
        np.testing.assert_allclose(float(l.detach()), float(f[f"loss{i}"].reshape(-1)[0]), rtol=1e-4)
    batch_loss = sum(losses)
    np.testing.assert_allclose(float(batch_loss.detach()), float(f["batch_loss"].reshape(-1)[0]), rtol=1e-4)
    batch_loss.backward()
    torch.cuda.synchronize()
    check_fixture_grads({k: p.grad for k, p in net.named_parameters()}, f, "config 3 union batch: ", step_atol=1e-6)
