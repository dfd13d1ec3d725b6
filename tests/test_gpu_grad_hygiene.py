"""Regressions for the weight-gradient reduction and the autograd/graph plumbing around it.

Round 1's scratch held one red run of test_net_small_forward_backward (block 1's
lin_proj.bias gradient garbage, 2.8 vs |ref| 1.4) that no committed tree reproduced.  The
suspects were (a) the shared ticket counters of the last-arriver colsum, (b) a partial-row
buffer a kernel leaves partly unwritten (fresh allocator memory is usually zero, reused memory
is not) and (c) a deferred weight-gradient sum AccumulateGrad adds to an existing .grad.  These
tests make each failure deterministic:
  - every torch.empty in the step starts from NaN-poisoned cached memory, repeatedly, and the
    gradients must match the reference fixture and be bitwise identical run to run;
  - concurrent column sums on two streams (each call now owns its counter range);
  - retain_graph double backward, and forward A / forward B / backward A / backward B
    (deferred sums must not be added to a .grad while unfilled);
  - CapturedStep after optimizer.zero_grad() (set_to_none) still delivers its gradients;
  - the PyG-call-form GATv2Conv never reuses the plan of a freed edge_index whose address a
    new, different edge_index got from the caching allocator.
"""
import numpy as np
import pytest
import torch

import gasfm_amd
from conftest import check_grad, golden
from gasfm_amd import _native

pytestmark = pytest.mark.gpu

OUT_ATOL, OUT_RTOL = 1e-4, 1e-3


def poison_cached_memory(device, mb=1024):
    """Fill the caching allocator's free blocks with NaN: later torch.empty calls in this process
    carve their buffers out of poisoned memory, so any element a kernel fails to write is NaN."""
    torch.cuda.synchronize(device)
    torch.cuda.empty_cache()
    keep = []
    for size in (512, 4096, 65536, 262144):  # small pool (<= 1 MB requests): 2 MB segments
        keep += [torch.full((size,), float("nan"), device=device) for _ in range(48)]
    keep.append(torch.full((mb << 18,), float("nan"), device=device))  # large pool
    torch.cuda.synchronize(device)
    del keep  # freed into the cache, not to the driver


def _scene(device):
    s = golden("scene_config1.npz")
    return gasfm_amd.SceneData(torch.from_numpy(s["M"]), torch.from_numpy(s["Ns"]), None, "config1").to(device)


def _net_small(device):
    f = golden("net_small.npz")
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.conf.small_conf(2))
    net.load_state_dict({k[3:]: torch.from_numpy(f[k]).float() for k in f.files if k.startswith("sd/")})
    return f, net.to(device)


def _loss(pred, f, device):
    return (pred["Ps_norm"] * torch.from_numpy(f["cP"]).float().to(device)).sum() + \
        (pred["pts3D"] * torch.from_numpy(f["cX"]).float().to(device)).sum()


def _grads(net):
    torch.cuda.synchronize()
    return {k: p.grad.detach().clone() for k, p in net.named_parameters()}


def test_poisoned_memory_repeated_steps_match_fixture_bitwise(device):
    data = _scene(device)
    f, net = _net_small(device)
    runs = []
    for it in range(3):
        poison_cached_memory(device)
        for p in net.parameters():
            p.grad = None
        pred = net(data)
        np.testing.assert_allclose(pred["Ps_norm"].detach().cpu().numpy(), f["Ps_norm"], atol=OUT_ATOL,
                                   rtol=OUT_RTOL)
        np.testing.assert_allclose(pred["pts3D"].detach().cpu().numpy(), f["pts3D"], atol=OUT_ATOL, rtol=OUT_RTOL)
        _loss(pred, f, device).backward()
        g = _grads(net)
        for k, v in g.items():
            check_grad(v, f["grad/" + k], f"run {it} {k}")
        runs.append(g)
    for k in runs[0]:
        assert torch.equal(runs[0][k], runs[1][k]) and torch.equal(runs[0][k], runs[2][k]), k


def test_poisoned_memory_scaled_config4(device):
    """A larger scene (split camera items, many workgroups, partial rows of every kind) under
    poisoned memory: finite gradients, bitwise identical to an unpoisoned run."""
    from gasfm_amd import synthetic
    sc = synthetic.scaled_config4(0.02, seed=7)
    data = gasfm_amd.SceneData.from_synthetic(sc, max_piece=64).to(device)
    torch.manual_seed(0)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3)).to(device)
    gen = torch.Generator().manual_seed(3)
    cP = torch.randn((sc.m, 3, 4), generator=gen).to(device)
    cX = torch.randn((4, sc.n), generator=gen).to(device)

    def step(poison):
        if poison:
            poison_cached_memory(device, mb=2048)
        for p in net.parameters():
            p.grad = None
        pred = net(data)
        ((pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX).sum()).backward()
        return _grads(net)

    ref = step(False)
    got = step(True)
    for k in ref:
        assert torch.isfinite(got[k]).all(), k
        assert torch.equal(ref[k], got[k]), k


def test_concurrent_colsums_on_two_streams(device):
    g = torch.Generator().manual_seed(11)
    As = [torch.randn(int(r), int(c), generator=g).to(device)
          for r, c in zip(torch.randint(100, 20000, (40,), generator=g), torch.randint(1, 700, (40,), generator=g))]
    ref = [A.double().sum(0) for A in As]
    streams = [torch.cuda.Stream(device), torch.cuda.Stream(device)]
    torch.cuda.synchronize()
    outs = [None] * len(As)
    for rep in range(3):
        for i, A in enumerate(As):
            with torch.cuda.stream(streams[i % 2]):
                outs[i] = _native.colsum(A)
        torch.cuda.synchronize()
        for i, (o, r) in enumerate(zip(outs, ref)):
            torch.testing.assert_close(o.double(), r, rtol=1e-5, atol=1e-3, msg=f"rep {rep} job {i}")


def test_counter_ranges_are_disjoint_between_calls(device):
    a = _native._counters(device, 5)
    b = _native._counters(device, 7)
    pa, pb = a.data_ptr(), b.data_ptr()
    assert pa + 5 * 4 <= pb or pb + 7 * 4 <= pa


def test_retain_graph_double_backward(device):
    data = _scene(device)
    f, net = _net_small(device)
    loss = _loss(net(data), f, device)
    loss.backward(retain_graph=True)
    g1 = _grads(net)
    loss.backward()
    g2 = _grads(net)
    for k in g1:
        assert torch.equal(g2[k], 2 * g1[k]), k
        check_grad(g1[k], f["grad/" + k], k)


def test_two_forwards_two_backwards(device):
    data = _scene(device)
    f, net = _net_small(device)
    la = _loss(net(data), f, device)
    lb = _loss(net(data), f, device)
    la.backward()
    ga = _grads(net)
    lb.backward()
    gb = _grads(net)
    for k in ga:
        check_grad(ga[k], f["grad/" + k], k)
        assert torch.equal(gb[k], 2 * ga[k]), k


def test_captured_step_survives_zero_grad(device):
    from gasfm_amd.graph_step import CapturedStep
    data = _scene(device)
    f, net = _net_small(device)

    cP = torch.from_numpy(f["cP"]).float().to(device)
    cX = torch.from_numpy(f["cX"]).float().to(device)

    def fwd_bwd():  # no host-to-device copies inside the captured step
        pred = net(data)
        loss = (pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX).sum()
        loss.backward()
        return loss

    step = CapturedStep(fwd_bwd, net.parameters(), warmup=1)
    assert step.captured, step.fallback_reason
    opt = torch.optim.SGD(net.parameters(), lr=0.0)
    for _ in range(2):
        opt.zero_grad()  # set_to_none=True (train.py:66)
        step()
        torch.cuda.synchronize()
        for k, p in net.named_parameters():
            assert p.grad is not None, k
            check_grad(p.grad, f["grad/" + k], k)


def test_pyg_call_form_plan_not_reused_across_tensors(device):
    """Two different edge_index tensors of the same shape at the same device address."""
    from gasfm_amd.gatv2 import GATv2Conv
    from oracle import pyg_gatv2
    torch.manual_seed(0)
    conv = GATv2Conv(16, 8, heads=2, add_self_loops=False).to(device)
    N, E = 50, 40
    x = torch.randn(N, 16, device=device)
    outs, refs = [], []
    for seed in (1, 2):
        g = torch.Generator().manual_seed(seed)
        src = torch.randperm(N, generator=g)[:E]
        dst = torch.randint(0, N, (E,), generator=g)
        ei = torch.stack([src, dst]).to(device)
        outs.append((ei.data_ptr(), conv(x, ei).detach().cpu()))
        ref = pyg_gatv2.GATv2Conv(16, 8, heads=2, add_self_loops=False).double()
        ref.load_state_dict({k: v.detach().cpu().double() for k, v in conv.state_dict().items()})
        refs.append(ref(x.cpu().double(), ei.cpu()).detach())
        del ei
    assert outs[0][0] == outs[1][0], "allocator did not reuse the address; the test needs it to"
    for (_, o), r in zip(outs, refs):
        torch.testing.assert_close(o.double(), r, rtol=1e-4, atol=1e-5)
