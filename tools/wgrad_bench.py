"""Weight-gradient products of the camera-row Linears: dense.splitk_wgrad (batched split-K slices +
an ordered column sum) against one dy^T x GEMM, per shape (R rows, M outputs, N inputs); per-call
time from 20 calls captured in one graph."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import dense  # noqa: E402


def _time(fn, reps=20, rounds=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(rounds):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * rounds)


def main():
    dev = torch.device("cuda:0")
    for R, M, N in ((1000, 1024, 4), (1000, 7, 1024), (1000, 1024, 32), (1000, 32, 1024), (125, 1024, 4),
                    (125, 7, 1024), (4000, 1024, 4), (16000, 64, 64)):
        dy, x = torch.randn(R, M, device=dev), torch.randn(R, N, device=dev)
        s = _time(lambda: dense.splitk_wgrad(dy, x))
        d = _time(lambda: dy.T @ x)
        print(json.dumps(dict(R=R, M=M, N=N, splitk_us=round(s, 2), direct_us=round(d, 2))), flush=True)


if __name__ == "__main__":
    main()
