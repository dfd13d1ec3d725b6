"""Do parallel branches of a captured hipGraph run concurrently on MI355X?

Captures 2 x 200 dependent tiny kernels either as one chain (one stream) or as two
independent chains (two streams forked from the capture stream) and times replays.
"""
import time

import torch


def chain(x, n):
    for _ in range(n):
        x = x + 1.0
    return x


def main():
    dev = torch.device("cuda", 0)
    a = torch.zeros(1024, device=dev)
    b = torch.zeros(1024, device=dev)
    n = 200
    for mode in ("serial", "two_streams"):
        g = torch.cuda.CUDAGraph()
        s2 = torch.cuda.Stream()
        chain(a, 2), chain(b, 2)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            if mode == "serial":
                oa = chain(a, n)
                ob = chain(b, n)
            else:
                cur = torch.cuda.current_stream()
                s2.wait_stream(cur)
                oa = chain(a, n)
                with torch.cuda.stream(s2):
                    ob = chain(b, n)
                cur.wait_stream(s2)
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        print(f"{mode}: {1e6 * dt / (2 * n):.2f} us per kernel ({1e3 * dt:.2f} ms per replay of {2 * n} kernels)",
              flush=True)


if __name__ == "__main__":
    main()
