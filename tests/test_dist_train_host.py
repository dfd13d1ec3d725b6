"""Host logic of the N-GPU config-5 step (gasfm_amd/dist_train.py), on the CPU: the point shards of a
scene cover its edges exactly once with the network's values (outlier-injected copy) and the loss's
values / pixel measurements (clean scene) on the same edges; the scene checksum that
ShardedTrainer(verify=True) all-reduces separates scenes that differ in one value."""
import numpy as np
import torch

from gasfm_amd import synthetic
from gasfm_amd.dist_train import scene_checksum, shard_device_scene
from gasfm_amd.scene import SceneData, SparseMat


def _scene(seed=3):
    sc = synthetic.windowed_scene(14, 900, mean_extra=4, seed=seed)
    return SceneData(torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns()), torch.from_numpy(sc.Ps_gt()), "s")


def _injected_copy(d):
    """The same edges with other values (what outlier injection hands the network)."""
    inp = SceneData.__new__(SceneData)
    inp.__dict__.update(d.__dict__)
    x = d.x
    inp.x = SparseMat(x.values + 0.25, x.indices, x.cam_per_pts, x.pts_per_cam, x.shape)
    return inp


def test_shards_cover_edges_with_both_value_sets():
    d = _scene()
    inp = _injected_copy(d)
    idx = d.x.indices.numpy()
    key = idx[0] * d.x.shape[1] + idx[1]
    for world in (1, 2, 3, 8):
        seen = []
        for r in range(world):
            net, loss = shard_device_scene(d, r, world, inp)
            p0 = net.point_slice.start
            li = net.x.indices.numpy()
            gk = li[0] * d.x.shape[1] + (li[1] + p0)
            pos = np.searchsorted(key, gk)
            assert np.array_equal(key[pos], gk)  # every local edge is an edge of the scene
            np.testing.assert_array_equal(net.x.values.numpy(), inp.x.values.numpy()[pos])
            np.testing.assert_array_equal(loss.x.values.numpy(), d.x.values.numpy()[pos])
            M = d._M.numpy()
            np.testing.assert_array_equal(loss.xy.numpy(), np.stack([M[2 * idx[0][pos], idx[1][pos]],
                                                                     M[2 * idx[0][pos] + 1, idx[1][pos]]], 1))
            assert net.n_edges_global == idx.shape[1] and loss.shard is net.shard
            seen.append(pos)
        allpos = np.concatenate(seen)
        assert np.array_equal(np.sort(allpos), np.arange(idx.shape[1]))  # each edge on exactly one rank


def test_scene_checksum_separates_scenes():
    d = _scene()
    a = scene_checksum(d)
    assert torch.equal(a, scene_checksum(_scene()))
    x = d.x
    vals = x.values.clone()
    vals[17, 1] = torch.nextafter(vals[17, 1], torch.tensor(10.0))
    d2 = SceneData.__new__(SceneData)
    d2.__dict__.update(d.__dict__)
    d2.x = SparseMat(vals, x.indices, x.cam_per_pts, x.pts_per_cam, x.shape)
    assert not torch.equal(a, scene_checksum(d2))
    assert not torch.equal(a, scene_checksum(_scene(seed=4)))
