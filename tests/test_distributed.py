"""Point-sharded multi-GPU path.

CPU (gloo, world size 2): sharding/plans, the collective wrappers, and the partial-softmax
decomposition the exchange relies on.  GPU: two ranks on one MI355X (gloo staging) must
reproduce the single-GPU forward and gradients.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gasfm_amd import distributed as gd
from gasfm_amd import synthetic


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_partition_points_balanced_and_covering():
    sc = synthetic.scaled_config4(0.02, seed=3)
    for world in (1, 2, 4, 8):
        b = gd.partition_points(sc.pt, sc.n, world)
        assert b[0] == 0 and b[-1] == sc.n and np.all(np.diff(b) >= 0)
        counts = np.bincount(sc.pt, minlength=sc.n)
        per = [counts[b[r]:b[r + 1]].sum() for r in range(world)]
        assert sum(per) == sc.num_edges
        assert max(per) - min(per) <= counts.max() + 1


def test_shard_scene_partitions_edges_and_replicates_views():
    sc = synthetic.scaled_config4(0.02, seed=3)
    world = 3
    shards = [gd.shard_scene(sc, r, world) for r in range(world)]
    assert sum(s.x.values.shape[0] for s in shards) == sc.num_edges
    glob_pt = np.concatenate([s.x.indices[1].numpy() + s.point_slice.start for s in shards])
    glob_cam = np.concatenate([s.x.indices[0].numpy() for s in shards])
    order = np.lexsort((glob_pt, glob_cam))
    np.testing.assert_array_equal(glob_cam[order], sc.cam)
    np.testing.assert_array_equal(glob_pt[order], sc.pt)
    v0 = shards[0].graph_wrappers["view2global"].plan
    for s in shards[1:]:
        v = s.graph_wrappers["view2global"].plan
        assert torch.equal(v.perm if v.perm is not None else torch.arange(v.num_edges, dtype=torch.int32),
                           v0.perm if v0.perm is not None else torch.arange(v0.num_edges, dtype=torch.int32))
    for s in shards:
        pp = s.partial_plans["proj2view"]
        assert pp.all_partial and pp.num_targets == sc.m


def test_local_param_classification():
    import gasfm_amd
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf())
    names = [k for k, _ in net.named_parameters()]
    local = [k for k in names if gd.is_local_param(k)]
    n_local = sum(p.numel() for k, p in net.named_parameters() if gd.is_local_param(k))
    assert "equivariant_blocks.3.global_feature_update.proj2view.graph_conv.att" in local
    assert "equivariant_blocks.3.global_feature_update.proj2view.graph_conv.lin_r.weight" not in local
    assert "view_head.0.weight" not in local and "scenepoint_head.4.bias" in local
    assert n_local < 1_000_000  # the bucket is ~1 MB of fp32, not the 145 M replicated params


def test_camera_rows_and_cam_param_classification():
    import gasfm_amd
    for m, world in ((1000, 8), (1000, 3), (10, 4)):
        rows = [gd.camera_rows(m, world, r) for r in range(world)]
        assert rows[0][0] == 0 and rows[-1][1] == m
        assert all(a[1] == b[0] for a, b in zip(rows[:-1], rows[1:]))
        assert all(r[2] == -(-m // world) for r in rows)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf())
    names = [k for k, _ in net.named_parameters()]
    part = {k for k in names if gd.is_local_param(k, cameras=True)}
    blk = "equivariant_blocks.3."
    # the view chain and every point-side parameter carry partial gradients ...
    for k in ("global_feature_update.proj2view.mlp.0.weight", "global_feature_update.proj2view.norm_and_proj_view2proj.2.weight",
              "global_feature_update.proj2view.graph_conv.lin_r.weight", "projection_feature_update.lin_view.weight",
              "global_feature_update.view_and_scenepoint2global.graph_conv_view2global.lin_l.weight",
              "global_feature_update.view_and_scenepoint2global.graph_conv_view2global.att",
              "projection_feature_update.lin_proj.weight"):
        assert blk + k in part, k
    assert "view_head.0.weight" in part and "scenepoint_head.4.bias" in part
    # ... the global chain does not
    for k in ("global_feature_update.view_and_scenepoint2global.mlp.0.weight",
              "global_feature_update.view_and_scenepoint2global.proj_view_and_scenepoint2global.weight",
              "global_feature_update.view_and_scenepoint2global.graph_conv_view2global.lin_r.weight",
              "projection_feature_update.lin_global.weight", "global_feature_update.proj2view.graph_conv.bias"):
        assert blk + k not in part, k
    # every point-sharding local parameter stays partial under camera sharding
    assert {k for k in names if gd.is_local_param(k)} <= part


def test_watchdog_retire_private_api_present():
    """graph_step.retire_collectives rests on two private torch.distributed symbols
    (c10d._world.pg_map, ProcessGroup._wait_for_pending_works): pinned on this torch, and a process
    group without the method makes it raise instead of silently skipping the retire step."""
    from gasfm_amd import graph_step
    assert graph_step.private_api_ok(), torch.__version__

    class _NoWait:  # a stand-in process group that lacks the private method
        pass

    import unittest.mock as um
    with um.patch.object(graph_step, "_process_groups", lambda: [_NoWait()]), \
            um.patch.object(dist, "is_initialized", lambda: True), \
            um.patch.object(dist, "get_backend", lambda pg: "nccl"):
        with pytest.raises(RuntimeError, match="_wait_for_pending_works"):
            graph_step.retire_collectives()


def _partial_state(logits, vals):
    m = logits.max(0).values
    e = torch.exp(logits - m)
    return m, e.sum(0), (e[:, :, None] * vals).sum(0)


def test_partial_softmax_merge_is_exact_decomposition():
    """What the exchange computes: per-rank (max, sum, acc) merged in rank order == full softmax."""
    g = torch.Generator().manual_seed(0)
    E, H, C = 97, 4, 8
    logits = torch.randn(E, H, generator=g, dtype=torch.float64) * 3
    vals = torch.randn(E, H, C, generator=g, dtype=torch.float64)
    full = torch.softmax(logits, 0)
    ref = (full[:, :, None] * vals).sum(0)
    cuts = [0, 10, 10, 60, E]  # includes an empty rank
    M = torch.full((H,), -float("inf"), dtype=torch.float64)
    S = torch.zeros(H, dtype=torch.float64)
    A = torch.zeros(H, C, dtype=torch.float64)
    for a, b in zip(cuts[:-1], cuts[1:]):
        if b == a:
            continue
        m, s, acc = _partial_state(logits[a:b], vals[a:b])
        mn = torch.maximum(M, m)
        f1 = torch.where(torch.isinf(M), torch.zeros_like(M), torch.exp(M - mn))
        f2 = torch.exp(m - mn)
        S, A, M = S * f1 + s * f2, A * f1[:, None] + acc * f2[:, None], mn
    torch.testing.assert_close(A / S[:, None], ref, rtol=1e-12, atol=1e-12)


def _worker_collectives(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = gd.ShardContext(rank, world)
        t = torch.full((3, 2), float(rank + 1))
        g = shard.all_gather(t)
        x = torch.ones(4, requires_grad=True)
        y = gd.AllReduceGrad.apply(x, shard)
        (y * (rank + 1)).sum().backward()
        # several tensors, one all-reduce; b's output is unused on rank 0 (None gradient)
        a = torch.ones(2, 3, requires_grad=True)
        b = torch.ones(5, requires_grad=True)
        ya, yb = gd.AllReduceGradN.apply(shard, a, b)
        ((ya * (rank + 1)).sum() + (yb.sum() * 10.0 if rank == 1 else 0.0)).backward()
        q.put((rank, g.tolist(), x.grad.tolist(), a.grad.tolist(), b.grad.tolist()))
    finally:
        dist.destroy_process_group()


def test_collective_wrappers_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_collectives, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, gr, ga, gb)) for r, g, gr, ga, gb in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        g, gr, ga, gb = res[r]
        assert g == [[1.0, 1.0]] * 3 + [[2.0, 2.0]] * 3  # rank-ordered gather
        assert gr == [3.0] * 4  # gradient summed over ranks (1 + 2)
        assert ga == [[3.0] * 3] * 2 and gb == [10.0] * 5  # AllReduceGradN: one all-reduce, None -> 0


def _worker_sharded_model(rank, world, port, q, cameras=False, bounds=None, max_piece=64):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gasfm_amd
        from oracle.weights import deterministic_state_dict
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        sc = synthetic.scaled_config4(0.02, seed=5)
        net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
        net.load_state_dict(deterministic_state_dict(net.state_dict()))
        model = gd.ShardedGraphAttnSfMNet(net.to(dev), cameras=cameras)
        data = gd.shard_scene(sc, rank, world, max_piece=max_piece, cameras=cameras, point_bounds=bounds).to(dev)
        g = torch.Generator().manual_seed(1)
        cP = torch.randn((sc.m, 3, 4), generator=g).to(dev)
        cX = torch.randn((4, sc.n), generator=g).to(dev)
        pred = model(data)
        loss = (pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX[:, data.point_slice]).sum()
        loss.backward()
        model.sync_grads()
        # numpy (pickled by value): tensors would travel as shared-memory fds owned by this process
        grads = {k: p.grad.detach().cpu().numpy() for k, p in net.named_parameters()}
        q.put((rank, pred["Ps_norm"].detach().cpu().numpy(), pred["pts3D"].detach().cpu().numpy(),
               (data.point_slice.start, data.point_slice.stop), grads))
    finally:
        dist.destroy_process_group()


def _run_sharded_vs_oracle(device, world, cameras, bounds=None, max_piece=64):
    """``world`` ranks (gloo staging, all on one GPU) vs the single-GPU forward, and both vs the fp64
    oracle's gradients; every parameter gradient bitwise identical across the ranks."""
    import gasfm_amd
    from conftest import check_grad, oracle_grads
    from oracle.weights import deterministic_state_dict
    sc = synthetic.scaled_config4(0.02, seed=5)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
    sd64 = deterministic_state_dict(net.state_dict(), torch.float64)
    net.load_state_dict({k: v.float() for k, v in sd64.items()})
    net = net.to(device)
    data = gasfm_amd.SceneData.from_synthetic(sc, max_piece=64).to(device)
    g = torch.Generator().manual_seed(1)
    cP = torch.randn((sc.m, 3, 4), generator=g).to(device)
    cX = torch.randn((4, sc.n), generator=g).to(device)
    pred = net(data)
    ((pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX).sum()).backward()
    (g64, _), (g32, _) = oracle_grads(sd64, sc, cP.cpu().double(), cX.cpu().double())

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_sharded_model, args=(r, world, port, q, cameras, bounds, max_piece))
             for r in range(world)]
    for p in procs:
        p.start()
    res = _collect(q, procs)
    res.sort(key=lambda t: t[0])
    assert [r[3] for r in res] == [(int(a), int(b)) for a, b in zip(res_bounds(sc, world, bounds)[:-1],
                                                                     res_bounds(sc, world, bounds)[1:])]
    for rank, ps, pts, (a, b), grads in res:
        np.testing.assert_allclose(ps, pred["Ps_norm"].detach().cpu().numpy(), atol=1e-5, rtol=1e-4)
        np.testing.assert_allclose(pts, pred["pts3D"][:, a:b].detach().cpu().numpy(), atol=1e-5, rtol=1e-4)
        for k in g64:
            check_grad(grads[k], g64[k], f"rank {rank} {k}", g32[k])
    for k, p in net.named_parameters():
        check_grad(p.grad, g64[k], f"single-GPU {k}", g32[k])
    # every parameter gradient ends bitwise identical on every rank (replicated optimizer steps stay in sync)
    for rank in range(1, world):
        for k in g64:
            assert np.array_equal(res[0][4][k], res[rank][4][k]), (rank, k)


def _collect(q, procs, timeout=600):
    """One result per process; fails at once when a rank dies (its peers would wait forever in a
    collective), terminating the rest."""
    import queue
    import time
    res, t0 = [], time.time()
    try:
        while len(res) < len(procs):
            try:
                res.append(q.get(timeout=2))
                continue
            except queue.Empty:
                pass
            dead = [i for i, p in enumerate(procs) if p.exitcode not in (None, 0)]
            assert not dead, f"rank(s) {dead} exited with {[procs[i].exitcode for i in dead]}"
            assert time.time() - t0 < timeout, "sharded ranks timed out"
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
    return res


def res_bounds(sc, world, bounds):
    return gd.partition_points(sc.pt, sc.n, world) if bounds is None else np.asarray(bounds)


@pytest.mark.gpu
@pytest.mark.parametrize("cameras", [False, True], ids=["points", "points+cameras"])
def test_sharded_model_matches_single_gpu(device, cameras):
    """2 ranks (gloo staging, one GPU) vs the single-GPU forward, and both vs the fp64 oracle's grads;
    points sharded, and points + camera rows sharded (the view chain split over the ranks)."""
    _run_sharded_vs_oracle(device, 2, cameras)


def _bounds_with_small_shard(world):
    """Edge-balanced point ranges except that rank 3 keeps only 5 points (a shard far smaller than a
    camera work item, next to ranks holding the rest)."""
    sc = synthetic.scaled_config4(0.02, seed=5)
    b = gd.partition_points(sc.pt, sc.n, world).copy()
    b[4] = b[3] + 5
    return b


@pytest.mark.gpu
@pytest.mark.parametrize("cameras,small", [(False, False), (True, False), (True, True)],
                         ids=["points", "points+cameras", "points+cameras-small-shard"])
def test_sharded_model_world8_matches_oracle(device, cameras, small):
    """The 8-way decomposition bench.py's N = 8 path takes: 8 gloo ranks on one GPU,
    scaled config 4 (m = 20, n = 4000), 3 blocks.  camera_rows(20, 8) gives ranks of 3, 2 and 0
    camera rows; eight partial rows per camera merge; the camera plans use the shard-sized piece
    length (camera_max_piece); small: one rank holds only 5 points."""
    bounds = _bounds_with_small_shard(8) if small else None
    _run_sharded_vs_oracle(device, 8, cameras, bounds=bounds, max_piece=None)


def _worker_capture_agree(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gasfm_amd
        from gasfm_amd.graph_step import CapturedStep
        from oracle.weights import deterministic_state_dict
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        sc = synthetic.scaled_config4(0.02, seed=5)
        net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=2))
        net.load_state_dict(deterministic_state_dict(net.state_dict()))
        model = gd.ShardedGraphAttnSfMNet(net.to(dev))
        data = gd.shard_scene(sc, rank, world, max_piece=64).to(dev)
        cP = torch.ones((sc.m, 3, 4), device=dev)
        cX = torch.ones((4, sc.n), device=dev)[:, data.point_slice].contiguous()

        def fwd_bwd():
            pred = model(data)
            loss = (pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX).sum()
            loss.backward()
            model.sync_grads()
            return loss

        def agree(ok):
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return bool(t.item())

        step = CapturedStep(fwd_bwd, net.parameters(), warmup=1, agree=agree)
        loss = step()
        g = net.equivariant_blocks[1].projection_feature_update.lin_proj.weight.grad
        q.put((rank, step.captured, step.fallback_reason, float(loss), g.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_capture_fallback_is_agreed_across_ranks(device):
    """gloo stages collectives through the host, so capture fails: every rank must fall back to
    eager together (a rank-local fallback would desynchronise the collectives) and still step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_capture_agree, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=600) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [False, False], [r[2] for r in res]
    assert np.array_equal(res[0][4], res[1][4])  # synced local-parameter gradient


@pytest.mark.gpu
@pytest.mark.parametrize("cams", [False, True], ids=["points", "points+cameras"])
def test_rccl_bench_captures_and_replays(tmp_path, cams):
    """bench.py's RCCL path (nccl process group, one rank) captures the whole step, collectives
    included, into a hipGraph and replays it.  Regression: in the default "global" capture mode
    ProcessGroupNCCL's watchdog thread querying events during the capture aborted the process."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(repo, "bench.py"),
           "--gpus", "1", "--dist", "--cameras", "200", "--points", "20000", "--layers", "2", "--steps", "3", "--warmup", "2",
           "--no-cpu-baseline"] + (["--cam-shard-1"] if cams else [])
    r = subprocess.run(cmd, cwd=repo, env=env, capture_output=True, text=True, timeout=110)
    (tmp_path / "bench_stderr.log").write_text(r.stderr)
    # the watchdog's what() (the HIP error it rethrew) sits far above the stack frames at the tail
    why = [ln for ln in r.stderr.splitlines()
           if "terminated with exception" in ln or "HIP error" in ln or "Error" in ln.split(":")[0]]
    assert r.returncode == 0, "\n".join(why[:12]) + "\n...\n" + r.stderr[-1500:]
    assert "hipGraph replay" in r.stderr, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["execution"].startswith("hipGraph replay") and res["value"] > 0
    # camera sharding: RCCL all-gathers of the view rows and the overlapped (async) weight-gradient
    # all-reduces, issued from post-accumulate-grad hooks, inside the captured graph
    assert ("point+camera" in res["config"]["parallelism"]) == cams


@pytest.mark.gpu
def test_captured_step_survives_watchdog_polls():
    """a step whose async all-reduce puts the process group's RCCL stream into the
    capture, held open 0.3 s so that ProcessGroupNCCL's watchdog polls (every 100 ms) during it,
    after warm-up steps that listed Works on the watchdog.  CapturedStep retires those Works before
    capturing (graph_step.retire_collectives), so no poll touches an event of a capturing stream."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "watchdog_capture_probe.py"), "--child", "D"],
                       cwd=repo, env=env, capture_output=True, text=True, timeout=110)
    why = [ln for ln in r.stderr.splitlines() if "terminated with exception" in ln or "HIP error" in ln]
    assert r.returncode == 0, "\n".join(why[:12]) + "\n...\n" + r.stderr[-1500:]
    assert "case D: captured True" in r.stdout, r.stdout


def _esfm_conf(valid_only=True):
    import gasfm_amd
    return gasfm_amd.Conf({"model": {"view_head": {"enabled": True}, "scenepoint_head": {"enabled": True}},
                           "loss": {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
                                    "normalize_grad_wrt_valid_projections_only": valid_only, "hinge_loss": True,
                                    "hinge_loss_weight": 1.0}})


def _worker_sharded_esfm(rank, world, port, q, valid_only=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gasfm_amd
        from oracle.weights import deterministic_state_dict
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        sc = synthetic.scaled_config4(0.02, seed=5)
        net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=2))
        net.load_state_dict(deterministic_state_dict(net.state_dict()))
        model = gd.ShardedGraphAttnSfMNet(net.to(dev))
        data = gd.shard_scene(sc, rank, world, max_piece=64).to(dev)
        loss = gasfm_amd.ESFMLoss(_esfm_conf(valid_only))(model(data), data)
        loss.backward()
        model.sync_grads()
        grads = {k: p.grad.detach().cpu().numpy() for k, p in net.named_parameters()}
        q.put((rank, float(loss), grads))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("valid_only", [True, False])
def test_sharded_esfm_loss_matches_single_gpu(device, valid_only):
    """ESFMLoss on a point-sharded scene: every rank gets the GLOBAL loss (sum and
    #valid-depth all-reduced, divided by the global edge count) and, after sync_grads, every
    parameter gradient equals the single-GPU one and is bitwise identical across ranks.
    valid_only=False: the equalized gradients divide by the GLOBAL edge count
    (loss_functions.py:110), not the rank's own."""
    import gasfm_amd
    from oracle.weights import deterministic_state_dict
    sc = synthetic.scaled_config4(0.02, seed=5)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=2))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    net = net.to(device)
    data = gasfm_amd.SceneData.from_synthetic(sc, max_piece=64).to(device)
    loss = gasfm_amd.ESFMLoss(_esfm_conf(valid_only))(net(data), data)
    loss.backward()
    ref = {k: p.grad.detach().double().cpu().numpy() for k, p in net.named_parameters()}

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_sharded_esfm, args=(r, 2, port, q, valid_only)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=600) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, l, grads in res:
        assert abs(l - float(loss)) <= 1e-5 * abs(float(loss)), (rank, l, float(loss))
        for k, r in ref.items():
            g = grads[k].astype(np.float64)
            nr = np.linalg.norm(r)
            assert np.linalg.norm(g - r) <= 1e-3 * nr + 1e-7, f"rank {rank} {k}: {np.linalg.norm(g - r):.3e} / {nr:.3e}"
    for k in ref:
        assert np.array_equal(res[0][2][k], res[1][2][k]), k


@pytest.mark.gpu
def test_bench_self_launches_n_ranks(tmp_path):
    """VERDICT r5 #1 end to end: ``python bench.py --gpus 2`` with no launcher in the environment starts
    two torchrun ranks itself (a child process), they run the sharded step and rank 0 prints ONE JSON
    line with n_gpus 2.  gloo on one GPU (RCCL cannot put two ranks on one device): the N-rank launch,
    rank logic and max-over-ranks timing, not the wire."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--backend", "gloo", "--one-gpu",
           "--cameras", "100", "--points", "10000", "--layers", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=repo, env=env, capture_output=True, text=True, timeout=240)
    (tmp_path / "bench_stderr.log").write_text(r.stderr)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["value"] > 0 and "x2" in res["config"]["parallelism"]
