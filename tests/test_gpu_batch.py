"""Several scenes in one forward (gasfm_amd/batch.py) against one forward per scene.

The union graph computes the per-scene forwards exactly (disjoint graphs, one global node per
scene, the global projection term folded into the per-camera term), so the bar is fp32
summation order: outputs |d| <= 1e-5 + 1e-4 |ref|; parameter gradients of the summed
per-scene losses elementwise rtol 1e-4, atol 1e-6 (12-block learning conf, training-step-sized scenes
sampled and augmented on the device as in train.py).
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from gasfm_amd import synthetic
from gasfm_amd.batch import SceneBatch, forward_batch
from gasfm_amd.conf import Conf
from gasfm_amd.loss import ESFMLoss
from gasfm_amd.scene_device import apply_rotational_homography_aug_device, sample_data_device, scene_from_dense_device

pytestmark = pytest.mark.gpu


def _scenes(device, k=3, views=(12, 15, 18)):
    np.random.seed(0)
    torch.manual_seed(0)
    out = []
    for i in range(k):
        sc = synthetic.windowed_scene(40, 3000, mean_extra=6, seed=20 + i)
        full = scene_from_dense_device(torch.from_numpy(sc.dense_M()).to(device), torch.from_numpy(sc.Ns()).to(device),
                                       torch.from_numpy(sc.Ps_gt()).to(device), f"s{i}")
        out.append(apply_rotational_homography_aug_device(sample_data_device(full, views[i % len(views)]), 15, 20))
    return out


def _conf():
    base = gasfm_amd.learning_conf()
    return Conf({"dataset": {"calibrated": True}, "model": base.d["model"],
                 "loss": {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
                          "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True,
                          "hinge_loss_weight": 1.0}})


def _grads(net):
    return [p.grad.detach().clone() if p.grad is not None else None for p in net.parameters()]


def test_batch_forward_backward_matches_per_scene(device):
    torch.manual_seed(1)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    lossf = ESFMLoss(conf)
    datas = _scenes(device)
    net.zero_grad(set_to_none=True)
    ref_pred = [net(d) for d in datas]
    sum(lossf(p, d) for p, d in zip(ref_pred, datas)).backward()
    g_ref = _grads(net)
    net.zero_grad(set_to_none=True)
    pred = forward_batch(net, datas)
    sum(lossf(p, d) for p, d in zip(pred, datas)).backward()
    g = _grads(net)
    for a, b in zip(pred, ref_pred):
        for k in ("Ps_norm", "pts3D"):
            np.testing.assert_allclose(a[k].detach().cpu().numpy(), b[k].detach().cpu().numpy(), rtol=1e-4, atol=1e-5)
    names = [n for n, _ in net.named_parameters()]
    for n, a, b in zip(names, g, g_ref):
        assert (a is None) == (b is None), n
        if a is None:
            continue
        # elementwise, as the several-forwards test: tiny cancellation-limited gradients (the
        # attention vectors' ~1e-7 entries) differ at fp32 summation-order level
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=n)


def test_batch_structure(device):
    datas = _scenes(device, k=2)
    b = SceneBatch(datas)
    M = sum(d.x.shape[0] for d in datas)
    assert b.x.shape[0] == M and b.scene_of_cam.shape[0] == M
    assert b.graph_wrappers["view2global"].plan.num_targets == 2
    assert b.graph_wrappers["scenepoint2global"].plan.num_targets == 2
    key = b.x.indices[0] * b.x.shape[1] + b.x.indices[1]
    assert bool((key[1:] > key[:-1]).all())  # still camera-major


def test_batch_reads_scene_build_arrays_without_building_graphs(device):
    """Device-built scenes build their graph wrappers on first use (scene_device, round 3): the union
    batch and ESFMLoss read the scene-build arrays, so no per-scene plan is built, and the union's
    plans -- hence the outputs -- are bitwise those of a batch built from the scenes' plans."""
    torch.manual_seed(2)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    lossf = ESFMLoss(conf)
    datas = _scenes(device)
    assert all("graph_wrappers" not in d.__dict__ for d in datas)
    with torch.no_grad():
        pred = forward_batch(net, datas)
        loss = sum(lossf(p, d) for p, d in zip(pred, datas))
    assert all("graph_wrappers" not in d.__dict__ for d in datas)
    lazy = SceneBatch(datas)
    for d in datas:
        d.graph_wrappers  # noqa: B018  (build them: SceneBatch then reads the plans)
    eager = SceneBatch(datas)
    for name in ("proj2view", "proj2scenepoint", "view2global", "scenepoint2global"):
        a, b = lazy.graph_wrappers[name].plan, eager.graph_wrappers[name].plan
        for k in ("seg_ptr", "items", "combine"):
            assert torch.equal(getattr(a, k).cpu(), getattr(b, k).cpu()), (name, k)
        assert (a.perm is None) == (b.perm is None) and (a.perm is None or torch.equal(a.perm.cpu(), b.perm.cpu()))
        assert (a.n_slots, a.n_items, a.n_part_rows) == (b.n_slots, b.n_items, b.n_part_rows)
    with torch.no_grad():
        pred2 = forward_batch(net, datas)
        loss2 = sum(lossf(p, d) for p, d in zip(pred2, datas))
    for p, q in zip(pred, pred2):
        assert torch.equal(p["Ps_norm"], q["Ps_norm"]) and torch.equal(p["pts3D"], q["pts3D"])
    assert torch.equal(loss, loss2)
