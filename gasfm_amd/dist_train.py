"""Config-5 training step on W GPUs: one sampled, augmented, outlier-injected scene per step,
point-sharded over the ranks (BASELINE.json configs[4]; train.py:49-152).

The GASFM learning confs train with ``dataset.batch_size = 1`` (learning_euc_rhaug-15-20_gasfm.conf:5,
multiple_scenes_learning.py:59-65): a step is ONE scene, sampled to 10-20 views, rotated (rhaug
15 / 20 degrees), with 10 % of its projections replaced by outliers for the network's input
(train.py:73-81, dataset_utils.py:430-461) and the clean measurements for the loss (train.py:82-90).
Here every rank makes that scene itself from the same training scene with the same seeded draws --
the sampling, augmentation and injection draws are numpy / torch CPU generators consumed in the
reference's order (scene_device.py, outliers.py) and the device passes are deterministic -- so the
W ranks hold bit-identical scenes without any transfer (``scene_checksum`` / ``verify=True`` asserts
it with one all-reduce).  Then per rank:

  shard_device_scene   the rank's contiguous point range (edge-balanced, distributed.partition_points)
                       with every edge of those points, cam-major as the reference's SparseMat; the
                       network's shard carries the injected values, the loss's the clean ones
  forward              distributed.ShardedGraphAttnSfMNet (camera partials all-gathered and merged in
                       rank order; view / global chains replicated)
  ESFMLoss             the global loss from (sum, #valid-depth) all-reduced; dPs all-reduced, dpts3D
                       rank-local (loss.ESFMLossFn)
  compute_core_errors  our_repro from the local edges' (sum, count), all-reduced
  sync_grads           one all-reduce of the rank-local parameters' gradients
  optimizer            gasfm_amd.optim.Adam (one launch): identical gradients on every rank give
                       bitwise identical weights, so no parameter broadcast is needed

``StaticTrainer`` (static_batch.py) is the single-GPU captured form of the same step; this module is
its point-sharded counterpart, run eagerly: the shard's plans are rebuilt per sampled scene on the
host from one device-to-host copy of the scene's edges.
"""
import copy

import numpy as np
import torch
import torch.distributed as dist

from . import _native
from .distributed import ShardContext, ShardedGraphAttnSfMNet, shard_scene
from .evaluation import _pixel_cameras, _pixel_measurements
from .scene import SparseMat


class _HostEdges:
    """The view of a device scene that distributed.shard_scene reads: m, n, cam-major (cam, pt) and
    the per-edge network input values (one device-to-host copy)."""

    def __init__(self, data, values=None):
        idx = data.x.indices.detach().to("cpu", torch.int64)
        self.cam, self.pt = idx[0].numpy(), idx[1].numpy()
        self.m, self.n = int(data.x.shape[0]), int(data.x.shape[1])
        v = data.x.values if values is None else values
        self._vals = v.detach().to("cpu", torch.float32).numpy()

    def normalized_values(self):
        return self._vals


def scene_checksum(data):
    """int64 [4] device tensor: (E, m, n, a position-weighted sum of the edge indices and of the value
    bit patterns).  Equal on every rank iff (barring collisions) the ranks built the same scene."""
    idx = data.x.indices.to(torch.int64)
    E = idx.shape[1]
    w = torch.arange(1, E + 1, dtype=torch.int64, device=idx.device)
    bits = data.x.values.detach().float().contiguous().view(torch.int32).to(torch.int64)
    h = ((idx[0] * 1000003 + idx[1]) * w).sum() + (bits.sum(1) * w).sum()
    return torch.stack([torch.tensor(E, device=idx.device), torch.tensor(int(data.x.shape[0]), device=idx.device),
                        torch.tensor(int(data.x.shape[1]), device=idx.device), h])


def shard_device_scene(data, rank, world, inputs=None, cameras=False, emulate=False, max_piece=None):
    """(network shard, loss shard) of a device scene for this rank.

    data: the clean scene (loss, errors); inputs: the network's scene with the same edges (outlier
    injection replaces values only), default ``data``.  Both shards live on data's device, share the
    plans and differ only in ``x.values``.  The loss shard also carries ``xy`` (pixel measurements of
    the local edges) and ``Ns`` for the per-step reprojection error."""
    inputs = data if inputs is None else inputs
    if inputs.x.indices.shape != data.x.indices.shape:
        raise ValueError("shard_device_scene: the network's input scene has other edges than the loss's")
    dev = data.x.values.device
    host = _HostEdges(data, inputs.x.values)
    net = shard_scene(host, rank, world, max_piece=max_piece, cameras=cameras, emulate=emulate).to(dev)
    p0, p1 = net.point_slice.start, net.point_slice.stop
    sel = np.nonzero((host.pt >= p0) & (host.pt < p1))[0]
    sel_d = torch.from_numpy(sel).to(dev)
    loss = copy.copy(net)
    xl = net.x
    loss.x = SparseMat(data.x.values.detach().float().index_select(0, sel_d).contiguous(), xl.indices,
                       xl.cam_per_pts, xl.pts_per_cam, xl.shape)
    loss.xy = _pixel_measurements(data).index_select(0, sel_d).contiguous()
    loss.Ns = data.Ns
    loss.Ns_invT = getattr(data, "Ns_invT", None)
    return net, loss


def sharded_repro_error(loss_shard, pred):
    """compute_core_errors' our_repro (evaluation.py:8-31) of a point-sharded scene: the local edges'
    (sum, count) of reprojection errors, all-reduced; 0-d device tensor (nan without valid depths)."""
    idx = loss_shard.x.indices
    cam, pt = idx[0].to(torch.int32).contiguous(), idx[1].to(torch.int32).contiguous()
    P = _pixel_cameras(loss_shard, pred["Ps_norm"])
    X = pred["pts3D"].detach().float().contiguous()
    tot = _native.colsum(_native.reproj_error(cam, pt, loss_shard.xy, P, X, None))
    tot = loss_shard.shard.all_reduce_(tot)
    return tot[0] / tot[1]


class ShardedTrainer:
    """One config-5 training step per call on this rank (module docstring).

    net: this rank's GraphAttnSfMNet (same initial weights on every rank); lossf: ESFMLoss;
    optimizer: stepped after sync_grads (gasfm_amd.optim.Adam keeps the ranks bitwise in step).
    group: the process group (default: the world); world / rank from it unless ``emulate_world``
    (one GPU standing in for rank 0 of that many: collectives become local copies, timing only)."""

    def __init__(self, net, lossf, optimizer=None, group=None, cameras=False, emulate_world=0, verify=False):
        self.net, self.lossf, self.optimizer = net, lossf, optimizer
        self.group = group
        self.cameras = cameras
        self.emulate_world = int(emulate_world)
        if self.emulate_world > 1:
            self.rank, self.world = 0, self.emulate_world
        else:
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.model = ShardedGraphAttnSfMNet(net, group=group, cameras=cameras)
        self.params = [p for p in net.parameters() if p.requires_grad]
        self.verify = verify
        self.last = None  # (net shard, loss shard) of the last step

    def _check_same_scene(self, *scenes):
        if self.emulate_world > 1:
            return
        for d in scenes:
            c = scene_checksum(d)
            lo, hi = c.clone(), c.clone()
            sh = ShardContext(self.rank, self.world, self.group)
            if sh._staged(c):
                lo, hi = lo.cpu(), hi.cpu()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
            if not torch.equal(lo, hi):
                raise RuntimeError("ShardedTrainer: the ranks built different scenes (seed the numpy / torch "
                                   "generators identically on every rank)")

    def step(self, data, inputs=None, errors=True):
        """data: the clean sampled + augmented scene; inputs: its outlier-injected copy (the network's
        input), default ``data``.  Returns (loss, our_repro) as 0-d device tensors (our_repro None with
        errors=False); leaves the summed gradients in p.grad and steps the optimizer."""
        inputs = data if inputs is None else inputs
        if self.verify:
            self._check_same_scene(data, inputs)
        net_shard, loss_shard = shard_device_scene(data, self.rank, self.world, inputs, cameras=self.cameras,
                                                   emulate=self.emulate_world > 1)
        self.last = (net_shard, loss_shard)
        for p in self.params:
            p.grad = None
        pred = self.model(net_shard)
        loss = self.lossf(pred, loss_shard)
        err = sharded_repro_error(loss_shard, pred) if errors else None
        loss.backward()
        self.model.sync_grads()
        if self.optimizer is not None:
            self.optimizer.step()
        return loss.detach(), err


def sample_training_scene(full, outlier_rate=0.1, inplane=15, tilt=20, views=None, log=lambda s: None):
    """(clean scene, network input scene) of one config-5 sample (train.py:60-81 with the
    rhaug-15-20 + outliers0.1 confs): 10-20 consecutive views (SceneData.sample_data), the rotational
    homography augmentation, then outlier injection for the network's copy (None when the injection's
    sampling failed, as the reference's inject_outliers returns None).  The draws come from numpy's
    global generator and torch's (CPU and device) generators: seed them identically on every rank."""
    from .outliers import inject_outliers
    from .scene_device import apply_rotational_homography_aug_device, sample_data_device
    v = int(np.random.randint(10, 21)) if views is None else int(views)
    d = apply_rotational_homography_aug_device(sample_data_device(full, v, build=False), inplane, tilt)
    if not outlier_rate:
        return d, d
    return d, inject_outliers(d, outlier_rate, log=log)
