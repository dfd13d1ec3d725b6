"""Device scene builder (scene_build.hip) vs the host builder on a config-4-sized dense M.

usage: python tools/scene_bench.py [m] [n] [--no-host]
Builds the dense [2m, n] measurement matrix of the config-4 synthetic scene on the GPU, then
times (HIP events, median of 5) each builder pass and the whole ``scene_from_dense_device``
against ``SceneData(M, Ns)`` on the host CPU (once).  Roofline: the mask pass streams M
(8 m n bytes) once; the emit / point-CSR passes touch the 1-bit mask (m n / 8 bytes) plus
O(E) outputs.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gasfm_amd  # noqa: E402
from gasfm_amd import _native, synthetic  # noqa: E402
from gasfm_amd.scene_device import scene_from_dense_device  # noqa: E402


def timed(fn, reps=5):
    ts = []
    out = None
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    m = int(args[0]) if args else 1000
    n = int(args[1]) if len(args) > 1 else 200_000
    dev = torch.device("cuda", 0)
    sc = synthetic.windowed_scene(m, n, seed=4)
    cam = torch.from_numpy(np.asarray(sc.cam, dtype=np.int64)).to(dev)
    pt = torch.from_numpy(np.asarray(sc.pt, dtype=np.int64)).to(dev)
    rng = np.random.default_rng(0)
    xy = torch.from_numpy(rng.uniform(1, 1000, size=(sc.num_edges, 2)).astype(np.float32)).to(dev)
    M = torch.zeros((2 * m, n), dtype=torch.float32, device=dev)
    M[2 * cam, pt] = xy[:, 0]
    M[2 * cam + 1, pt] = xy[:, 1]
    K = np.array([[800, 0, 500], [0, 800, 500], [0, 0, 1]], dtype=np.float64)
    Ns = torch.from_numpy(np.repeat(np.linalg.inv(K)[None], m, 0).astype(np.float32)).to(dev)
    E = sc.num_edges
    print(f"m={m} n={n} E={E}  dense M {M.numel() * 4 / 1e9:.2f} GB", flush=True)

    L = _native.lib()
    W, T = L.gasfm_scene_mask_words(n), L.gasfm_scene_tiles(m, n)
    i32 = dict(dtype=torch.int32, device=dev)
    mask = torch.empty(m * W, dtype=torch.int64, device=dev)
    pv = torch.empty(W, dtype=torch.int64, device=dev)
    vc, pc = torch.empty(n, **i32), torch.empty(n, **i32)
    tc, tb = torch.empty(T, **i32), torch.empty(T + 1, **i32)
    st = _native._stream(M)
    p = _native._p

    def mask_pass():
        _native.check(L.gasfm_scene_mask(p(M), M.stride(0), m, n, p(mask), p(vc), p(pv), p(pc), p(tc), p(tb), st),
                      "mask")
    ms_mask, _ = timed(mask_pass)
    bytes_mask = M.numel() * 4 + mask.numel() * 8 + n * 12
    print(f"scene_mask (+ptvalid, tilecount, scan): {ms_mask * 1e3:8.1f} us  "
          f"{bytes_mask / ms_mask / 1e6:7.0f} GB/s of {bytes_mask / 1e9:.2f} GB algorithmic", flush=True)
    assert int(tb[T]) == E, (int(tb[T]), E)
    ms_all, s = timed(lambda: scene_from_dense_device(M, Ns))
    print(f"scene_from_dense_device (all passes + 4 plans, incl. host syncs): {ms_all:8.2f} ms", flush=True)
    assert s.x.values.shape[0] == E
    if "--no-host" not in sys.argv:
        Mc, Nc = M.cpu(), Ns.cpu()
        t0 = time.perf_counter()
        h = gasfm_amd.SceneData(Mc, Nc, None, "host")
        dt = time.perf_counter() - t0
        print(f"host SceneData(M, Ns) on {torch.get_num_threads()} CPU threads: {dt * 1e3:8.1f} ms", flush=True)
        assert torch.equal(h.x.indices, s.x.indices.cpu())
        assert torch.equal(h.graph_wrappers["proj2scenepoint"].plan.perm, s.graph_wrappers[
            "proj2scenepoint"].plan.perm.cpu())
        print("device == host: indices, point perm", flush=True)


if __name__ == "__main__":
    main()
