"""Per-launch time of the global GATv2 kernels (csrc/global_attn.hip) by problem mix and size:
views only, points only, both, forward (sharded partial rows and full outputs) and backward.
Each case: 20 launches captured in one graph, replayed 10 times, HIP events around the replays."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import _native  # noqa: E402

H, SLOPE = 4, 0.2


def _prob(rows, HC, dev, gen, part):
    r = lambda *s: torch.randn(*s, generator=gen, device="cpu").to(dev)  # noqa: E731
    d = dict(XL=r(rows, HC), src=None, S=rows, XR=r(HC), att=r(HC) * HC ** -0.5 * 2, bias=r(HC) * 0.1)
    if part:
        d["part"] = torch.empty(HC + 2 * H, device=dev)
    else:
        d.update(out=torch.empty(HC, device=dev), smax=torch.empty(H, device=dev), ssum=torch.empty(H, device=dev))
    return d


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, nargs="+", default=[125, 1000])
    ap.add_argument("--points", type=int, nargs="+", default=[25000, 200000])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(0)
    for nv, npt in zip(args.views, args.points):
        for mix in ("views", "points", "both"):
            for part in (True, False):
                probs = []
                if mix in ("views", "both"):
                    probs.append(_prob(nv, 1024, dev, gen, part))
                if mix in ("points", "both"):
                    probs.append(_prob(npt, 64, dev, gen, part))
                us = _time(lambda: _native.gatt_fwd(probs, SLOPE))
                print(json.dumps(dict(dir="fwd", mix=mix, views=nv, points=npt, part=part, us=round(us, 2))), flush=True)
            probs = []
            if mix in ("views", "both"):
                probs.append(_prob(nv, 1024, dev, gen, False))
            if mix in ("points", "both"):
                probs.append(_prob(npt, 64, dev, gen, False))
            _native.gatt_fwd(probs, SLOPE)
            for d in probs:
                HC = d["XL"].shape[1]
                d.update(gout=torch.randn(HC, device=dev), dXL=torch.empty_like(d["XL"]),
                         dXR=torch.empty(HC, device=dev), datt=torch.empty(2 * HC, device=dev))
            us = _time(lambda: _native.gatt_bwd(probs, SLOPE))
            print(json.dumps(dict(dir="bwd", mix=mix, views=nv, points=npt, us=round(us, 2))), flush=True)


if __name__ == "__main__":
    main()
