"""Generate full-width TRAINING-STEP gradient fixtures from the REFERENCE's own code (build container only).

    python tests/golden/make_golden_grads.py

The reference's GraphAttnSfMNet (models/graph_attn_sfm.py), SceneData (datasets/SceneData.py) and
ESFMLoss (loss_functions.py:69-123) are imported in place (tests/golden/refimport.py; PyG's GATv2Conv
is the oracle restatement, the only stand-in).  Weights: oracle/weights.py (deterministic per key).
Every run is float64 (and float32 for the fp32 reference-error bound).

  net_optim9_grads.npz    config 2 (single-scene optimisation, optim_euc_gasfm.conf: 9 blocks,
                          full width, its loss section) on a windowed 40-view x 1500-point scene:
                          M, Ns, outputs, loss, and every parameter gradient.
  train_step12.npz        config 3 (multi-scene learning step, learning_euc conf: 12 blocks) as
                          train.py:60-134 runs it: a batch of two scenes (12 and 17 views),
                          batch_loss = sum of the scenes' ESFMLoss, one backward.

Gradients of tensors with more than 256 elements are stored as projections G.reshape(rows, -1) @ r
(rows = the first dimension, or 16 for a vector) with r = oracle.weights.probe_vector(key, cols)
(regenerable), the rest in full.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refimport  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402  (input generation only)
from make_golden import conf_dict  # noqa: E402
from oracle.pyg_gatv2 import GATv2Conv as OracleGATv2Conv  # noqa: E402
from oracle.weights import deterministic_state_dict  # noqa: E402

LOSS = {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
        "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True, "hinge_loss_weight": 1.0}
FULL_MAX = 256


class _CpuMaskTaggedCuda(torch.Tensor):
    """The reference asserts data.valid_pts.is_cuda (loss_functions.py:122) only to dodge a CPU
    nonzero bug; the CPU mask reads is_cuda True so the unmodified reference runs on the CPU."""

    @property
    def is_cuda(self):
        return True


def grad_record(name, g):
    from oracle.weights import probe_vector
    g = g.detach().double()
    if g.numel() <= FULL_MAX:
        return {name: g.numpy()}
    rows = g.shape[0] if g.dim() >= 2 else (16 if g.numel() % 16 == 0 else 1)
    G = g.reshape(rows, -1)
    r = torch.from_numpy(probe_vector(name.split("/", 1)[1], G.shape[1]))
    return {name + "@r": (G @ r).numpy()}


def project_all(prefix, grads):
    out = {}
    for k, g in grads.items():
        out.update(grad_record(f"{prefix}/{k}", g))
    return out


def scene(ref, m, n, seed, dtype):
    sc = synthetic.windowed_scene(m, n, seed=seed)
    M, Ns = torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns())
    data = ref.SceneData.SceneData(M, Ns, torch.from_numpy(sc.Ps_gt()), f"windowed{m}x{n}", calibrated=True)
    data.x.values = data.x.values.to(dtype)
    feed = type("Data", (), {})()
    feed.norm_M = data.norm_M.to(dtype)
    feed.valid_pts = data.valid_pts.as_subclass(_CpuMaskTaggedCuda)
    return M, Ns, data, feed


def train_step(ref, conf, sd, scenes, dtype):
    """train.py:60-134 for one batch: zero_grad, sum of per-scene losses, one backward."""
    torch.manual_seed(0)
    net = ref.graph_attn_sfm.GraphAttnSfMNet(conf).to(dtype)
    net.load_state_dict({k: v.to(dtype) for k, v in sd.items()})
    lossf = ref.loss_functions.ESFMLoss(conf)
    batch_loss = torch.zeros(1, dtype=dtype)
    preds = []
    for data, feed in scenes:
        pred = net(data)
        loss = lossf(pred, feed).as_subclass(torch.Tensor)
        batch_loss = batch_loss + loss
        preds.append((pred["Ps_norm"].detach(), pred["pts3D"].detach(), loss.detach()))
    batch_loss.backward()
    return preds, batch_loss.detach(), {k: p.grad for k, p in net.named_parameters()}


def main():
    ref = refimport.load(OracleGATv2Conv)
    torch.set_grad_enabled(True)

    # config 2: optim conf, 9 blocks
    conf = conf_dict(9, 1024, 2048)
    conf.d["loss"] = dict(LOSS)
    template = ref.graph_attn_sfm.GraphAttnSfMNet(conf).state_dict()
    sd = deterministic_state_dict(template, torch.float64)
    out = {}
    for dt, tag in ((torch.float64, ""), (torch.float32, "_fp32")):
        M, Ns, data, feed = scene(ref, 40, 1500, 21, dt)
        preds, loss, grads = train_step(ref, conf, sd, [(data, feed)], dt)
        out.update({f"Ps_norm{tag}": preds[0][0].numpy(), f"pts3D{tag}": preds[0][1].numpy(),
                    f"loss{tag}": loss.numpy()})
        out.update(project_all("grad" + tag, grads))
        out["M"], out["Ns"] = M.float().numpy(), Ns.numpy()
        print(tag or "fp64", "loss", float(loss), "edges", data.x.values.shape[0])
    np.savez_compressed(os.path.join(HERE, "net_optim9_grads.npz"), **out)

    # config 3: learning conf, 12 blocks, a batch of two scenes
    conf = conf_dict(12, 1024, 2048)
    conf.d["loss"] = dict(LOSS)
    template = ref.graph_attn_sfm.GraphAttnSfMNet(conf).state_dict()
    sd = deterministic_state_dict(template, torch.float64)
    out = {}
    for dt, tag in ((torch.float64, ""), (torch.float32, "_fp32")):
        built = [scene(ref, m, n, s, dt) for m, n, s in ((12, 600, 31), (17, 900, 32))]
        preds, loss, grads = train_step(ref, conf, sd, [(d, f) for _, _, d, f in built], dt)
        for i, (M, Ns, _, _) in enumerate(built):
            out[f"M{i}"], out[f"Ns{i}"] = M.float().numpy(), Ns.numpy()
            out[f"loss{i}{tag}"] = preds[i][2].numpy()
        out[f"batch_loss{tag}"] = loss.numpy()
        out.update(project_all("grad" + tag, grads))
        print(tag or "fp64", "batch loss", float(loss))
    np.savez_compressed(os.path.join(HERE, "train_step12.npz"), **out)


if __name__ == "__main__":
    main()
