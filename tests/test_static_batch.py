"""Structure of the padded shape-stable union batch (gasfm_amd/static_batch.py), on the CPU.

Host-built scenes (SceneData's host builder) are filled into a bucket and every invariant the
kernels rely on is checked on the resulting buffers: cam-major edges, the real scenes' edges /
measurements / CSRs copied with their offsets, non-empty pieces tiling every camera, point and
scene segment, the combine entries and two-level rows covering exactly the slots, the pad scene's
degree bounds (cameras valid, points valid and unsplit), the scene maps and the loss weights; and
the bucket policy (a batch reuses a bucket it fits, a larger one does not fit).
"""
import numpy as np
import pytest
import torch

from gasfm_amd import static_batch, synthetic
from gasfm_amd.scene import SceneData


@pytest.fixture()
def small_pieces(monkeypatch):
    monkeypatch.setattr(static_batch, "S2G_PIECES", 64)


def _scenes(k=3, m0=12, n=1500):
    out = []
    for i in range(k):
        sc = synthetic.windowed_scene(m0 + 2 * i, n, mean_extra=4, seed=30 + i)
        out.append(SceneData(torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns()), torch.from_numpy(sc.Ps_gt()),
                             f"s{i}"))
    return out


def _tiles(items, lo, hi):
    """items (rows [seg, begin, end, ...]) tile [lo, hi) in order with non-empty pieces."""
    assert items[0, 1] == lo and items[-1, 2] == hi
    assert (items[:, 2] > items[:, 1]).all()
    assert (items[1:, 1] == items[:-1, 2]).all()


def test_static_batch_structure(small_pieces):
    datas = _scenes()
    st = static_batch.BatchStats(datas)
    assert st.expressible() is None
    caps = static_batch.Caps.for_batch(st)
    mp, npd, ep, dI = caps.pad(st)
    sb = static_batch.StaticBatch(caps, torch.device("cpu"))
    sb.fill(datas, st)
    M, N, E, S, B = caps.M, caps.N, caps.E, caps.S, caps.B
    cam, pt = sb.cam32.numpy(), sb.pt32.numpy()
    assert (np.diff(cam) >= 0).all() and cam[-1] == M - 1 and pt.max() == N - 1
    assert (sb.indices[0].numpy() == cam).all() and (sb.indices[1].numpy() == pt).all()
    mo, no, eo = sb.offsets
    for s, d in enumerate(datas):
        idx = d.x.indices.numpy()
        assert (cam[eo[s]:eo[s + 1]] == idx[0] + mo[s]).all() and (pt[eo[s]:eo[s + 1]] == idx[1] + no[s]).all()
        assert torch.equal(sb.values[eo[s]:eo[s + 1]], d.x.values.float())
    assert (sb.values[st.E:] == 0).all()
    # camera CSR and the all-split camera plan
    cptr = sb.cam_ptr.numpy().astype(np.int64)
    assert cptr[0] == 0 and cptr[-1] == E and (np.bincount(cam, minlength=M) == np.diff(cptr)).all()
    items = sb.items_c.numpy().astype(np.int64)
    assert items.shape == (caps.I, 4) and (items[:, 3] == np.arange(caps.I)).all()
    _tiles(items, 0, E)
    assert (np.diff(items[:, 0]) >= 0).all()
    comb = sb.comb_c.numpy()
    assert (comb[:, 0] == np.arange(M)).all() and (comb[:, 3] == 1).all()
    for c in range(M):
        rows = items[comb[c, 1]:comb[c, 1] + comb[c, 2]]
        assert (rows[:, 0] == c).all() and rows[0, 1] == cptr[c] and rows[-1, 2] == cptr[c + 1]
        if c < st.M:  # real cameras: the eager plans' pieces
            assert comb[c, 2] == max(1, -(-(cptr[c + 1] - cptr[c]) // static_batch.PIECE))
    # pad cameras valid (>= 8 edges), >= 1 piece, one camera of scene B each
    degc = np.diff(cptr)[st.M:]
    assert len(degc) == mp and degc.min() >= 8 and comb[st.M:, 2].sum() == dI
    # point CSR, perm / pos, the unsplit point plan
    pptr = sb.pt_ptr.numpy().astype(np.int64)
    perm, pos = sb.perm.numpy(), sb.pos.numpy()
    assert (np.sort(perm) == np.arange(E)).all() and (pos[perm] == np.arange(E)).all()
    assert (pt[perm] == np.repeat(np.arange(N), np.diff(pptr))).all()
    for p0 in (0, st.N - 1, st.N, N - 1):  # edges of a point in increasing edge order (stable CSR)
        assert (np.diff(perm[pptr[p0]:pptr[p0 + 1]]) > 0).all()
    ip = sb.items_p.numpy()
    assert (ip[:, 0] == np.arange(N)).all() and (ip[:, 3] == -1).all()
    _tiles(ip, 0, E)
    degp = np.diff(pptr)[st.N:]
    assert len(degp) == npd and degp.min() >= 2 and degp.max() <= static_batch.PIECE
    assert (sb.cam_per_pts.view(-1).numpy() == np.diff(pptr)).all()
    assert (sb.pts_per_cam.view(-1).numpy() == np.diff(cptr)).all()
    # scene maps, edge offsets, loss weights
    soc, sop = sb.soc32.numpy(), sb.sop32.numpy()
    assert (soc == np.repeat(np.arange(S), st.ms + [mp])).all() and (sb.scene_of_cam.numpy() == soc).all()
    assert (sop == np.repeat(np.arange(S), st.ns + [npd])).all()
    assert (sb.eoff.numpy() == np.array(eo + [E])).all()
    assert sb.weight.tolist() == [1.0] * B + [0.0]
    assert (soc[cam] == np.repeat(np.arange(S), np.diff(sb.eoff.numpy()))).all()
    # view2global: PV pieces per scene over its valid views, every scene split, one combine entry each
    src_v, seg_v = sb.src_v.numpy(), sb.seg_v.numpy()
    valid_v = np.diff(cptr) >= 8
    assert (src_v == np.nonzero(valid_v)[0]).all()
    assert (np.diff(seg_v) == np.bincount(soc[valid_v], minlength=S)).all()
    iv, PV = sb.items_v.numpy(), caps.PV
    assert iv.shape == (S * PV, 4) and (iv[:, 3] == np.arange(S * PV)).all()
    _tiles(iv, 0, seg_v[-1])
    for s in range(S):
        assert (iv[s * PV:(s + 1) * PV, 0] == s).all() and iv[s * PV, 1] == seg_v[s]
        assert tuple(sb.comb_v.numpy()[s]) == (s, s * PV, PV, 1)
    # scenepoint2global: P pieces per scene, all split, fixed two-level combine
    src_p, seg_p = sb.src_p.numpy(), sb.seg_p.numpy()
    valid_p = np.diff(pptr) >= 2
    assert (src_p == np.nonzero(valid_p)[0]).all()
    assert (np.diff(seg_p) == np.bincount(sop[valid_p], minlength=S)).all()
    its = sb.items_s.numpy()
    P = caps.P
    assert its.shape == (S * P, 4) and (its[:, 3] == np.arange(S * P)).all()
    _tiles(its, 0, seg_p[-1])
    for s in range(S):
        assert (its[s * P:(s + 1) * P, 0] == s).all() and its[s * P, 1] == seg_p[s]
    l1, cs = sb.l1_s.numpy(), sb.comb_s.numpy()
    assert (l1[:, 0] == S * P + np.arange(S * caps.NG)).all()
    for s in range(S):
        rows = l1[s * caps.NG:(s + 1) * caps.NG]
        assert rows[0, 1] == s * P and (rows[1:, 1] == rows[:-1, 1] + rows[:-1, 2]).all()
        assert rows[:, 2].sum() == P
        assert tuple(cs[s]) == (s, S * P + s * caps.NG, caps.NG, 1)
    # the host-side restatement of the global plans the GPU fill copies in (all views / points valid)
    assert (sb._host_plans(st, npd) == sb.hostfed.numpy()).all()
    plans = {n: w.plan for n, w in sb.graph_wrappers.items()}
    assert plans["proj2view"].n_slots == caps.I and plans["proj2view"].n_combine == M
    assert plans["scenepoint2global"].n_part_rows == S * P + S * caps.NG


def test_bucket_reuse_and_fit(small_pieces):
    datas = _scenes()
    st = static_batch.BatchStats(datas)
    caps = static_batch.Caps.for_batch(st)
    assert caps.pad(st) is not None and caps.waste_ok(st)
    # a batch of two of the three scenes fits the three-scene bucket's sizes only with B = 3
    st2 = static_batch.BatchStats(datas[:2])
    assert caps.pad(st2) is None
    # a slightly smaller batch of three reuses the bucket; the same scenes grown do not fit
    smaller = static_batch.BatchStats(_scenes(m0=11, n=1450))
    assert caps.pad(smaller) is not None
    bigger = static_batch.BatchStats(_scenes(m0=14, n=1700))
    assert caps.pad(bigger) is None
    # the sizes a new bucket gets for the bigger batch fit it
    assert static_batch.Caps.for_batch(bigger).pad(bigger) is not None


def test_inv3():
    A = torch.randn(5, 3, 3, dtype=torch.float64) + 3 * torch.eye(3, dtype=torch.float64)
    torch.testing.assert_close(static_batch._inv3(A), torch.linalg.inv(A))


def test_trainer_bucket_lru(small_pieces, monkeypatch):
    """StaticTrainer keeps at most max_buckets buckets, dropping the least recently used."""
    trainer = static_batch.StaticTrainer.__new__(static_batch.StaticTrainer)
    trainer.buckets, trainer.max_buckets = {}, 2
    monkeypatch.setattr(static_batch, "StaticBatch", lambda caps, dev: type("SB", (), {"caps": caps})())
    sts = [static_batch.BatchStats(_scenes(m0=m, n=n)) for m, n in ((8, 900), (12, 1500), (16, 2100))]
    keys = []
    for st in sts:
        b, new = trainer._bucket(st, torch.device("cpu"))
        assert new
        keys.append(b[0].caps.key())
    assert list(trainer.buckets) == keys[1:]  # the first (least recently used) was dropped
    b, new = trainer._bucket(sts[1], torch.device("cpu"))  # reuse moves it to the end
    assert not new and list(trainer.buckets) == [keys[2], keys[1]]


@pytest.mark.parametrize("m", [8, 10, 13, 16, 20])
def test_one_scene_batch_gets_a_bucket(small_pieces, m):
    """B = 1 (the GASFM learning confs' batch_size): a batch of one 8-20 view scene gets a bucket with
    >= V2G_PIECES pad cameras (round 6: 13 views gave 3 pad cameras and Caps.for_batch never
    returned), and the padded structure holds (test_static_batch_structure's invariants on B = 1)."""
    sc = synthetic.windowed_scene(m, 1500, mean_extra=4, seed=40 + m)
    datas = [SceneData(torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns()), torch.from_numpy(sc.Ps_gt()), "s")]
    st = static_batch.BatchStats(datas)
    assert st.expressible() is None
    caps = static_batch.Caps.for_batch(st)
    pad = caps.pad(st)
    assert pad is not None and pad[0] >= static_batch.V2G_PIECES and caps.waste_ok(st)
    sb = static_batch.StaticBatch(caps, torch.device("cpu"))
    sb.fill(datas, st)
    _tiles(sb.items_c[:, :3].numpy(), 0, caps.E)
    assert int(sb.cam_ptr[-1]) == caps.E and int(sb.pt_ptr[-1]) == caps.E
