"""The shape-stable union batch (gasfm_amd/static_batch.py) against the eager union batch (batch.py).

The padded bucket runs the real scenes' computation of the eager union with a disjoint, zero-weight
pad scene, every camera through a partial slot, other global-graph pieces and per-scene loss partials:
fp32 summation order only.  Bars (as tests/test_gpu_batch.py): outputs |d| <= 1e-5 + 1e-4 |ref|, the
loss and the per-scene reprojection errors rtol 1e-5, parameter gradients elementwise rtol 1e-4,
atol 1e-6.  In the trainer tests a few cancellation-limited weight-gradient entries differ by up to
~4e-6 (up to ~7e-4 relative with config 5's outliers: the global graphs' other piece lengths change
the order of their softmax sums, and large loss gradients cancel in the column sums), so there a
gradient tensor passes elementwise as above OR norm-wise, ||diff|| <= 1e-3 ||ref||; the replay
itself is checked against the same padded computation run eagerly: loss rtol 1e-6, gradients
rtol 1e-4 / atol 1e-7 (not bitwise: a library GEMM may pick another algorithm inside a capture).  The trainer test replays a bucket captured on one batch with ANOTHER batch's data
filled into its static buffers -- the captured graph must read everything it depends on from them.
12-block learning conf, training-step-sized scenes sampled and augmented on the device.
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from gasfm_amd import evaluation, static_batch, synthetic
from gasfm_amd.batch import forward_batch
from gasfm_amd.loss import ESFMLoss
from gasfm_amd.scene_device import apply_rotational_homography_aug_device, sample_data_device, scene_from_dense_device

from test_gpu_batch import _conf, _grads

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def s2g_pieces(monkeypatch):
    monkeypatch.setattr(static_batch, "S2G_PIECES", 128)  # the test scenes have ~1-2k valid points


def _scenes(device, views, seed=0, n=3000):
    np.random.seed(seed)
    torch.manual_seed(seed)
    out = []
    for i, v in enumerate(views):
        sc = synthetic.windowed_scene(40, n, mean_extra=6, seed=20 + i + 7 * seed)
        full = scene_from_dense_device(torch.from_numpy(sc.dense_M()).to(device), torch.from_numpy(sc.Ns()).to(device),
                                       torch.from_numpy(sc.Ps_gt()).to(device), f"s{i}")
        out.append(apply_rotational_homography_aug_device(sample_data_device(full, v), 15, 20))
    return out


def _eager(net, lossf, datas):
    net.zero_grad(set_to_none=True)
    pred = forward_batch(net, datas)
    loss = sum(lossf(p, d) for p, d in zip(pred, datas))
    loss.backward()
    errs = [float(evaluation.reprojection_error_mean(d, p)) for p, d in zip(pred, datas)]
    return pred, float(loss), _grads(net), errs


def _check_grads(net, g, g_ref, normwise=False):
    """Elementwise rtol 1e-4, atol 1e-6; normwise: a tensor also passes when ||a - b|| <= 1e-3 ||b||."""
    for (n, _), a, b in zip(net.named_parameters(), g, g_ref):
        assert (a is None) == (b is None), n
        if a is None:
            continue
        if normwise and float((a.double() - b.double()).norm()) <= 1e-3 * float(b.double().norm()):
            continue
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6, msg=lambda m: f"{n}: {m}")


def test_static_batch_matches_eager_union(device):
    torch.manual_seed(1)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    lossf = ESFMLoss(conf)
    datas = _scenes(device, (12, 15, 18))
    pred_ref, loss_ref, g_ref, err_ref = _eager(net, lossf, datas)
    st = static_batch.BatchStats(datas)
    assert st.expressible() is None
    sb = static_batch.StaticBatch(static_batch.Caps.for_batch(st), device)
    sb.fill(datas, st)
    net.zero_grad(set_to_none=True)
    pred = net(sb)
    loss = static_batch.batch_loss(pred, sb, lossf)
    tot = static_batch.batch_repro_errors(pred, sb)
    loss.backward()
    for a, b in zip(sb.split(pred), pred_ref):
        for k in ("Ps_norm", "pts3D"):
            np.testing.assert_allclose(a[k].detach().cpu().numpy(), b[k].detach().cpu().numpy(), rtol=1e-4, atol=1e-5)
    assert torch.isfinite(pred["Ps_norm"]).all() and torch.isfinite(pred["pts3D"]).all()  # the pad scene too
    assert abs(float(loss) - loss_ref) <= 1e-5 * abs(loss_ref)
    t = tot.tolist()
    np.testing.assert_allclose([a / b for a, b in t[:st.B]], err_ref, rtol=1e-5)
    _check_grads(net, _grads(net), g_ref)


def test_native_fill_matches_torch_fill(device):
    """gasfm_union_fill_scene / _pad + the host-fed global plans write exactly what fill_torch writes
    (Ns^-1: fp64 inverse vs the fp32 closed form, rtol 1e-5)."""
    from gasfm_amd.outliers import inject_outliers
    datas = _scenes(device, (12, 15, 18), seed=4)
    inputs = [inject_outliers(d, 0.1, log=lambda s: None) for d in datas]
    st = static_batch.BatchStats(inputs)
    caps = static_batch.Caps.for_batch(st)
    a, b = static_batch.StaticBatch(caps, device), static_batch.StaticBatch(caps, device)
    a.fill(datas, st, inputs)
    b.fill_torch(datas, st, inputs)
    for k in ("values", "values_loss", "xy", "indices", "cam32", "pt32", "cam_ptr", "pt_ptr", "perm", "pos",
              "cam_per_pts", "pts_per_cam", "scene_of_cam", "soc32", "sop32", "items_c", "comb_c", "items_p",
              "hostfed", "src_v", "src_p"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    torch.testing.assert_close(a.Ns_inv, b.Ns_inv, rtol=1e-5, atol=1e-6)


def test_static_trainer_replays_another_batch(device, monkeypatch):
    monkeypatch.setattr(static_batch, "MAX_WASTE", 10.0)  # the second batch reuses the first one's bucket
    torch.manual_seed(2)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    lossf = ESFMLoss(conf)
    trainer = static_batch.StaticTrainer(net, lossf)
    batches = [_scenes(device, (14, 16, 18), seed=0), _scenes(device, (10, 12, 13), seed=1)]
    for k, datas in enumerate(batches):
        loss, errs = trainer.step(datas)
        g = _grads(net)
        assert trainer.fallbacks == [] and trainer.eager_steps == 0
        assert len(trainer.buckets) == 1 and trainer.captures == 1
        sb, step = next(iter(trainer.buckets.values()))[:2]
        assert step.captured
        # the replay equals the same padded computation run eagerly on the buffers fill() wrote
        # (a stale input in the graph would show here at O(1))
        net.zero_grad(set_to_none=True)
        pred = net(sb)
        loss_st = static_batch.batch_loss(pred, sb, lossf)
        loss_st.backward()
        assert abs(float(loss) - float(loss_st)) <= 1e-6 * abs(float(loss_st)), k
        for (n, _), a, b in zip(net.named_parameters(), g, _grads(net)):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-7, msg=lambda m: f"{n}: {m}")
        _, loss_ref, g_ref, err_ref = _eager(net, lossf, datas)
        assert abs(float(loss) - loss_ref) <= 1e-5 * abs(loss_ref), k
        np.testing.assert_allclose(errs, err_ref, rtol=1e-5)
        _check_grads(net, g, g_ref, normwise=True)


def test_static_trainer_outlier_inputs(device):
    """Config 5: the network sees the outlier-injected scenes, the loss and errors the clean ones."""
    from gasfm_amd.outliers import inject_outliers
    torch.manual_seed(3)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    lossf = ESFMLoss(conf)
    datas = _scenes(device, (14, 16, 18), seed=2)
    inputs = [inject_outliers(d, 0.1, log=lambda s: None) for d in datas]
    assert all(x is not None for x in inputs)
    trainer = static_batch.StaticTrainer(net, lossf)
    loss, errs = trainer.step(datas, inputs)
    g = _grads(net)
    net.zero_grad(set_to_none=True)
    pred = forward_batch(net, inputs)
    loss_ref = sum(lossf(p, d) for p, d in zip(pred, datas))
    loss_ref.backward()
    err_ref = [float(evaluation.reprojection_error_mean(d, p)) for p, d in zip(pred, datas)]
    assert abs(float(loss) - float(loss_ref)) <= 1e-5 * abs(float(loss_ref))
    np.testing.assert_allclose(errs, err_ref, rtol=1e-5)
    _check_grads(net, g, _grads(net), normwise=True)


def test_static_trainer_prefetch_stream(device):
    """The pipelined use (tools/train_step_bench.py --pipeline): the batch and its BatchStats made on a
    second stream, the step on the main stream with read_errors=False; same loss, errors and
    gradients as the eager union."""
    torch.manual_seed(4)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    lossf = ESFMLoss(conf)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        datas = _scenes(device, (11, 14, 17), seed=5)
        st = static_batch.BatchStats(datas)
    torch.cuda.current_stream().wait_stream(side)
    trainer = static_batch.StaticTrainer(net, lossf)
    loss, err = trainer.step(datas, stats=st, read_errors=False)
    assert torch.is_tensor(err) and tuple(err.shape) == (3, 2)
    errs = trainer.errors(err)
    g = _grads(net)
    _, loss_ref, g_ref, err_ref = _eager(net, lossf, datas)
    assert abs(float(loss) - loss_ref) <= 1e-5 * abs(loss_ref)
    np.testing.assert_allclose(errs, err_ref, rtol=1e-5)
    _check_grads(net, g, g_ref, normwise=True)


def test_static_trainer_eager_fallback(device, monkeypatch):
    """A batch the padding cannot express runs through the eager union (counted, reason kept), with
    the same loss / errors / gradients, and the optimizer still steps."""
    from gasfm_amd.optim import Adam
    monkeypatch.setattr(static_batch, "S2G_PIECES", 10 ** 6)  # no scene has that many valid points
    torch.manual_seed(6)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    lossf = ESFMLoss(conf)
    datas = _scenes(device, (12, 15), seed=7)
    _, loss_ref, g_ref, err_ref = _eager(net, lossf, datas)
    before = [p.detach().clone() for p in net.parameters()]
    trainer = static_batch.StaticTrainer(net, lossf, optimizer=Adam(net.parameters(), lr=1e-3))
    loss, errs = trainer.step(datas)
    assert trainer.eager_steps == 1 and trainer.captures == 0 and "valid points" in trainer.fallbacks[0]
    assert abs(float(loss) - loss_ref) <= 1e-6 * abs(loss_ref)
    np.testing.assert_allclose(errs, err_ref, rtol=1e-6)
    _check_grads(net, _grads(net), g_ref)
    assert any(not torch.equal(p, b) for p, b in zip(net.parameters(), before))  # Adam stepped


def test_static_trainer_bf16_shadows_follow_the_optimizer(device, monkeypatch):
    """Config-5 bf16 mode under capture: after an optimizer step the replayed graph must read the new
    weights' bf16 shadows (StaticTrainer re-rounds them after the step).  A replay on the updated
    weights equals the eager union on them (rtol 1e-4); with stale shadows the lr = 1e-2 step would
    show at the percent level."""
    from gasfm_amd.optim import Adam
    monkeypatch.setattr(static_batch, "MAX_WASTE", 10.0)  # both batches in one bucket
    torch.manual_seed(8)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    net.set_projection_precision("bf16")
    lossf = ESFMLoss(conf)
    trainer = static_batch.StaticTrainer(net, lossf, optimizer=Adam(net.parameters(), lr=1e-2))
    a, b = _scenes(device, (14, 16, 18), seed=9), _scenes(device, (12, 13, 15), seed=10)
    trainer.step(a)  # capture, then Adam + shadow refresh
    trainer.optimizer = None  # the next replay leaves the weights as they are
    loss, _ = trainer.step(b)
    assert trainer.captures == 1 and trainer.eager_steps == 0
    net.zero_grad(set_to_none=True)
    ref = sum(lossf(p, d) for p, d in zip(forward_batch(net, b), b))
    assert abs(float(loss) - float(ref)) <= 1e-4 * abs(float(ref)), (float(loss), float(ref))
    # every live shadow equals its weight rounded to bf16 after the trainer's step (the refresh), and
    # a step without the refresh leaves them behind the weights (the check above is then needed)
    from gasfm_amd import dense

    def shadows_current():
        live = [(r(), sh) for r, sh, _, _ in dense._SHADOWS.values() if r() is not None]
        assert live
        return all(torch.equal(sh, w.detach().to(torch.bfloat16)) for w, sh in live)

    trainer.optimizer = Adam(net.parameters(), lr=1e-2)
    trainer.step(a)
    assert shadows_current()
    monkeypatch.setattr(net, "refresh_weight_shadows", lambda: None)
    trainer.step(a)
    assert not shadows_current()
    # an eager forward re-rounds the changed weights by itself (gasfm Adam bumps their versions)
    forward_batch(net, b)
    assert shadows_current()


def test_static_trainer_bf16_shadows_after_eager_fallback(device, monkeypatch):
    """the eager-fallback optimizer step re-rounds the bf16 shadows too.  Expressible batch
    (captured), then a batch that falls back to the eager union, then the captured bucket again: after
    each step every live shadow equals its weight in bf16, and the last replay equals the eager union
    on the updated weights."""
    from gasfm_amd import dense
    from gasfm_amd.optim import Adam
    monkeypatch.setattr(static_batch, "MAX_WASTE", 10.0)
    torch.manual_seed(12)
    conf = _conf()
    net = gasfm_amd.GraphAttnSfMNet(conf).to(device)
    net.set_projection_precision("bf16")
    lossf = ESFMLoss(conf)
    trainer = static_batch.StaticTrainer(net, lossf, optimizer=Adam(net.parameters(), lr=1e-2))
    a, b = _scenes(device, (14, 16, 18), seed=13), _scenes(device, (12, 13, 15), seed=14)

    def shadows_current():
        live = [(r(), sh) for r, sh, _, _ in dense._SHADOWS.values() if r() is not None]
        assert live
        return all(torch.equal(sh, w.detach().to(torch.bfloat16)) for w, sh in live)

    trainer.step(a)
    assert trainer.captures == 1 and shadows_current()
    monkeypatch.setattr(static_batch, "S2G_PIECES", 10 ** 6)
    trainer.step(b)  # the eager fallback, then Adam
    assert trainer.eager_steps == 1
    assert shadows_current()
    monkeypatch.setattr(static_batch, "S2G_PIECES", 128)
    trainer.optimizer = None
    loss, _ = trainer.step(a)  # the bucket captured on step 1, replayed on the new weights
    assert trainer.captures == 1
    net.zero_grad(set_to_none=True)
    ref = sum(lossf(p, d) for p, d in zip(forward_batch(net, a), a))
    assert abs(float(loss) - float(ref)) <= 1e-4 * abs(float(ref)), (float(loss), float(ref))
