"""CPU-side cost of issuing one training step vs its GPU time (GPU box).

Times (a) the host time to enqueue forward+backward with no synchronisation, and (b) the
synchronised step, on config 4 and on a 1/8-points scene (the per-rank load at 8 GPUs).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gasfm_amd  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402
from gasfm_amd.graph_step import CapturedStep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for n in (200_000, 25_000):
        sc = synthetic.windowed_scene(1000, n, seed=4)
        net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf()).to(dev)
        data = gasfm_amd.SceneData.from_synthetic(sc).to(dev)
        cP = torch.randn((sc.m, 3, 4), device=dev)
        cX = torch.randn((4, sc.n), device=dev)

        def step():
            p = net(data)
            ((p["Ps_norm"] * cP).sum() + (p["pts3D"] * cX).sum()).backward()
            for q in net.parameters():
                q.grad = None
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            step()
        t_enq = (time.perf_counter() - t0) / 5
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / 5
        print(f"n={n} E={sc.num_edges}: eager: host enqueue {1e3 * t_enq:.1f} ms/step, "
              f"wall {1e3 * t_all:.1f} ms/step", flush=True)

        def fwd_bwd():
            p = net(data)
            loss = (p["Ps_norm"] * cP).sum() + (p["pts3D"] * cX).sum()
            loss.backward()
            return loss
        cs = CapturedStep(fwd_bwd, net.parameters())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            cs()
        t_enq = (time.perf_counter() - t0) / 10
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / 10
        print(f"n={n} E={sc.num_edges}: graph ({'captured' if cs.captured else cs.fallback_reason}): "
              f"host enqueue {1e3 * t_enq:.2f} ms/step, wall {1e3 * t_all:.1f} ms/step", flush=True)


if __name__ == "__main__":
    main()
