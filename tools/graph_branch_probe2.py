"""Do independent branches of a captured hipGraph run concurrently on this ROCm?

Two chains of small kernels (1000x1024 fp32 adds, ~5 us each): serial on one stream vs
forked onto two / four streams inside the capture. Prints replay ms for each.
"""
import time
import torch


def run(nstreams, chain=200, rows=1000):
    dev = torch.device("cuda", 0)
    xs = [torch.randn(rows, 1024, device=dev) for _ in range(4)]
    main = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(4)]

    def body():
        if nstreams == 1:
            for i in range(4 * chain):
                xs[i % 4].add_(1.0)
            return
        cur = torch.cuda.current_stream()
        for s in side[:nstreams]:
            s.wait_stream(cur)
        for b in range(4):
            with torch.cuda.stream(side[b % nstreams]):
                for _ in range(chain):
                    xs[b].add_(1.0)
        for s in side[:nstreams]:
            cur.wait_stream(s)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        body()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            body()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t) / 10 * 1e3
    # eager
    with torch.cuda.stream(main):
        body()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            body()
        torch.cuda.synchronize()
    te = (time.perf_counter() - t) / 5 * 1e3
    print(f"streams={nstreams} rows={rows} kernels={4*chain}: graph {tg:.2f} ms, eager {te:.2f} ms", flush=True)


if __name__ == "__main__":
    for rows in (1000, 100):
        for ns in (1, 2, 4):
            run(ns, rows=rows)
