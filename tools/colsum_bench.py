"""colsum GPU time (graph replay) on the partial-buffer shapes the backward produces (GPU box)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import _native  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for rows, cols in ((4096, 64), (7168, 64), (125, 2048), (98, 128), (768, 2176), (512, 4288), (1000, 32),
                       (1024, 1088), (2048, 2176)):
        A = torch.randn(rows, cols, device=dev)

        def graph_time(fn):  # GPU time per call: 50 calls captured in one graph, replayed
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(50):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) * 1e3 / 50
        t = graph_time(lambda: _native.colsum(A))
        t2 = graph_time(lambda: A.sum(0))
        print(f"colsum {rows}x{cols}: {t:.1f} us  (torch sum(0): {t2:.1f} us)", flush=True)


if __name__ == "__main__":
    main()
