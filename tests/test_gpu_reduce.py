"""gasfm_colsum: one-launch deterministic column sums (last-arriver reduction) vs fp64."""
import pytest
import torch

from gasfm_amd import _native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(0, 7), (1, 1), (3, 5), (127, 64), (128, 64), (7168, 64), (2048, 2176),
                                       (100, 4288), (50_000, 36), (300, 1025)])
def test_colsum_matches_fp64_and_is_deterministic(device, rows, cols):
    g = torch.Generator().manual_seed(rows + 7 * cols)
    A = torch.randn(rows, cols, generator=g, dtype=torch.float64)
    ref = A.sum(0)
    Ad = A.float().to(device)
    outs = [_native.colsum(Ad) for _ in range(3)]  # repeated: the ticket counters must reset
    torch.testing.assert_close(outs[0].double().cpu(), ref, rtol=1e-5, atol=1e-5 * max(1, rows) ** 0.5)
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_colsum_strided_rows(device):
    A = torch.randn(999, 80, device=device)
    torch.testing.assert_close(_native.colsum(A[:, :64]), A[:, :64].sum(0), rtol=1e-5, atol=1e-4)


def test_colsum_multi_bitwise_equals_colsum(device):
    """One gasfm_colsum_multi launch over 60 jobs (two launches of <= 48) == 60 gasfm_colsum calls."""
    import ctypes
    g = torch.Generator().manual_seed(5)
    shapes = [(int(r), int(c)) for r, c in zip(torch.randint(0, 3000, (60,), generator=g),
                                                torch.randint(1, 3000, (60,), generator=g))]
    As = [torch.randn(r, c, generator=g).to(device) for r, c in shapes]
    ref = [_native.colsum(A) for A in As]
    L = _native.lib()
    n = len(As)
    ws = [torch.empty(int(L.gasfm_colsum_ws_floats(r, c)), device=device) for r, c in shapes]
    out = [torch.full((c,), float("nan"), device=device) for _, c in shapes]
    arr = lambda ty, xs: (ty * n)(*xs)  # noqa: E731
    cols = arr(ctypes.c_int32, [c for _, c in shapes])
    cnt = _native._counters(torch.device(device), L.gasfm_colsum_multi_counters(n, cols))
    for _ in range(2):  # the counters must reset
        st = L.gasfm_colsum_multi(n, arr(ctypes.c_void_p, [a.data_ptr() for a in As]),
                                  arr(ctypes.c_int64, [r for r, _ in shapes]), cols,
                                  arr(ctypes.c_int64, [c for _, c in shapes]),
                                  arr(ctypes.c_void_p, [w.data_ptr() for w in ws]),
                                  arr(ctypes.c_void_p, [o.data_ptr() for o in out]), _native._p(cnt),
                                  _native._stream(out[0]))
        assert st == 0, _native.lib().gasfm_last_error()
        torch.cuda.synchronize()
        for a, b in zip(out, ref):
            assert torch.equal(a, b)


def test_batched_weight_grads_bitwise_equal_immediate(device):
    """GraphAttnSfMNet: the end-of-backward batched weight-gradient sums give the same bits as the
    immediate ones, and a second backward (accumulating into existing .grad) stays correct."""
    import gasfm_amd
    from gasfm_amd import synthetic
    from oracle.weights import deterministic_state_dict
    sc = synthetic.scaled_config4(0.02, seed=3)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(device)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=3))
    net.load_state_dict(deterministic_state_dict(net.state_dict()))
    net = net.to(device)
    g = torch.Generator().manual_seed(2)
    cP = torch.randn((sc.m, 3, 4), generator=g).to(device)
    cX = torch.randn((4, sc.n), generator=g).to(device)

    def grads(batch, twice=False):
        net.batch_weight_grads = batch
        for p in net.parameters():
            p.grad = None
        for _ in range(2 if twice else 1):
            pred = net(data)
            ((pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX).sum()).backward()
        torch.cuda.synchronize()
        return {k: p.grad.clone() for k, p in net.named_parameters()}

    imm, bat = grads(False), grads(True)
    assert not _native._PENDING, "a batch was left unflushed"
    for k in imm:
        assert torch.equal(imm[k], bat[k]), k
    acc_imm, acc_bat = grads(False, twice=True), grads(True, twice=True)
    for k in imm:
        assert torch.equal(acc_imm[k], acc_bat[k]), k
        torch.testing.assert_close(acc_bat[k], 2 * imm[k], rtol=1e-5, atol=1e-6)
    net.batch_weight_grads = True


@pytest.mark.parametrize("rows,cols", [(0, 2), (1, 2), (5, 3), (4097, 1), (4001638, 2), (200_000, 64),
                                       (200_000, 3), (12_345, 256), (99_999, 12), (300_000, 7)])
def test_colsum_tall_matches_fp64_and_is_deterministic(device, rows, cols):
    """gasfm_colsum_tall (bias gradients over E edge / n point rows) vs fp64, repeated bitwise."""
    assert _native.colsum_tall_ok(torch.empty(1, cols, device=device))
    g = torch.Generator().manual_seed(rows + 3 * cols)
    A = torch.randn(rows, cols, generator=g, dtype=torch.float64)
    ref = A.sum(0)
    Ad = A.float().to(device)
    outs = [_native.colsum_tall(Ad) for _ in range(3)]
    torch.testing.assert_close(outs[0].double().cpu(), ref, rtol=1e-5, atol=1e-5 * max(1, rows) ** 0.5)
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_colsum_tall_in_captured_graph(device):
    """Replayed from a hipGraph (where torch's global sum reduction was measured wrong), the
    tall column sum equals the eager one on every replay."""
    A = torch.randn(500_000, 2, device=device)
    eager = _native.colsum_tall(A)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _native.colsum_tall(A)
    torch.cuda.current_stream().wait_stream(s)
    from gasfm_amd.graph_step import gc_paused
    g = torch.cuda.CUDAGraph()
    with gc_paused(), torch.cuda.graph(g):
        out = _native.colsum_tall(A)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
