"""The captured training step (static_batch.StaticTrainer: padded bucket, one replayed hipGraph of
forward + ESFMLoss + backward) checked DIRECTLY against the reference, not through the eager union
(VERDICT r5 #3 / weak #5):

  (a) B = 2: train_step12.npz's two scenes (the reference's own GraphAttnSfMNet + ESFMLoss + summed
      batch loss, tests/golden/make_golden_grads.py) -> loss and every parameter gradient against the
      fixture at test_gpu_train_step.py's eager bars (check_fixture_grads: normwise 1e-3 or 10x the
      fp32 reference's own error, floor 1e-6 x the step's largest gradient norm) -- no extra escape;
  (b) B = 1, the GASFM learning confs' dataset.batch_size (learning_euc_rhaug-15-20_gasfm.conf:5,
      multiple_scenes_learning.py:59-65): one scene sampled and augmented on the device, the captured
      step's loss and gradients against the fp64 oracle on the same edges (test_gpu_train_step.py's
      device-data-path bars), and fixture scene 1 alone against its fixture loss.
Both require that the step was captured and replayed (no eager fallback).
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from conftest import check_fixture_grads, check_grad, golden, project_grad
from gasfm_amd import static_batch
from gasfm_amd.loss import ESFMLoss
from oracle.weights import deterministic_state_dict
from test_gpu_train_step import conf_with_loss, grads_of, net_for, scene

pytestmark = pytest.mark.gpu


def _captured_step(trainer, datas):
    loss, errs = trainer.step(datas)
    assert trainer.eager_steps == 0 and trainer.fallbacks == [], trainer.fallbacks
    assert trainer.captures == 1
    sb, step = next(iter(trainer.buckets.values()))[:2]
    assert step.captured
    return loss, errs


def test_static_trainer_b2_matches_reference_fixture(device, monkeypatch):
    monkeypatch.setattr(static_batch, "S2G_PIECES", 64)  # the fixture scenes have a few hundred valid points
    f = golden("train_step12.npz")
    conf = conf_with_loss(gasfm_amd.learning_conf())
    net = net_for(conf, device)
    trainer = static_batch.StaticTrainer(net, ESFMLoss(conf))
    datas = [scene(f[f"M{i}"], f[f"Ns{i}"], device, f"s{i}") for i in range(2)]
    loss, errs = _captured_step(trainer, datas)
    np.testing.assert_allclose(float(loss), float(f["batch_loss"].reshape(-1)[0]), rtol=1e-4)
    assert all(np.isfinite(errs))
    check_fixture_grads(grads_of(net), f, "captured B=2: ", step_atol=1e-6)
    # a second replay of the same bucket (the timed regime) gives the same loss and gradients
    g1 = {k: v.clone() for k, v in grads_of(net).items()}
    loss2, _ = trainer.step(datas)
    assert trainer.captures == 1
    np.testing.assert_allclose(float(loss2), float(loss), rtol=1e-6)
    for k, v in grads_of(net).items():
        torch.testing.assert_close(v, g1[k], rtol=1e-6, atol=1e-9, msg=lambda m: f"{k}: {m}")


def test_static_trainer_b1_fixture_scene_loss(device, monkeypatch):
    monkeypatch.setattr(static_batch, "S2G_PIECES", 64)
    f = golden("train_step12.npz")
    conf = conf_with_loss(gasfm_amd.learning_conf())
    net = net_for(conf, device)
    trainer = static_batch.StaticTrainer(net, ESFMLoss(conf))
    loss, _ = _captured_step(trainer, [scene(f["M1"], f["Ns1"], device, "s1")])
    np.testing.assert_allclose(float(loss), float(f["loss1"].reshape(-1)[0]), rtol=1e-4)


def test_static_trainer_b1_matches_fp64_oracle(device, monkeypatch):
    from gasfm_amd import synthetic
    from gasfm_amd.scene_device import apply_rotational_homography_aug_device, sample_data_device, \
        scene_from_dense_device
    from oracle import esfm_loss, gasfm_ref, scenes
    monkeypatch.setattr(static_batch, "S2G_PIECES", 128)
    np.random.seed(21)
    torch.manual_seed(21)
    conf = conf_with_loss(gasfm_amd.learning_conf())
    net = net_for(conf, device)
    sc = synthetic.windowed_scene(40, 2500, seed=61)
    full = scene_from_dense_device(torch.from_numpy(sc.dense_M()).to(device), torch.from_numpy(sc.Ns()).to(device),
                                   torch.from_numpy(sc.Ps_gt()).to(device), "train_b1")
    d = apply_rotational_homography_aug_device(sample_data_device(full, int(np.random.randint(10, 21))), 15, 20)
    trainer = static_batch.StaticTrainer(net, ESFMLoss(conf))
    loss, errs = _captured_step(trainer, [d])
    assert np.isfinite(errs[0])
    got = grads_of(net)

    refs = {}
    idx = d.x.indices.cpu().numpy()
    g = scenes.graph_from_edges(idx[0], idx[1], d.x.shape[0], d.x.shape[1])
    for dt in (torch.float64, torch.float32):
        sd = {k: v.clone().requires_grad_(True) for k, v in deterministic_state_dict(net.state_dict(), dt).items()}
        vals = d.x.values.detach().to(dt).cpu()
        r = gasfm_ref.forward(sd, vals, g, dtype=dt)
        total = esfm_loss.esfm_loss_edges(r["Ps_norm"], r["pts3D"], g.cam, g.pt, vals, 1e-4, True, 1.0, True, True)
        total.backward()
        refs[dt] = (float(total.detach()), {k: (v.grad if v.grad is not None else torch.zeros_like(v))
                                            for k, v in sd.items()})
    l64, l32 = refs[torch.float64][0], refs[torch.float32][0]
    np.testing.assert_allclose(float(loss), l64, rtol=max(1e-4, 10 * abs(l32 - l64) / abs(l64)))
    r64 = {k: project_grad(k, v) for k, v in refs[torch.float64][1].items()}
    floor = 1e-6 * max(np.linalg.norm(v) for v in r64.values()) + 1e-9
    for k, gv in got.items():
        check_grad(project_grad(k, gv), r64[k], k, project_grad(k, refs[torch.float32][1][k]), atol=floor)
