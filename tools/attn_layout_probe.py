"""A/B of the XL layout for the 32-wide attention kernels on the config-4 plans (GPU box).

usage: python tools/attn_layout_probe.py [--reps R]
XL interleaved [E, 64] (both directions' halves in one row, ld 64: what the prologue writes today)
vs contiguous [E, 32] per direction (ld 32).  Every launch is timed alone with HIP events, after
a 1 GiB write that evicts L2 / MALL (the in-step condition: XL was written by the prologue
~0.5 GB earlier), and also back to back (cache-warm).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gasfm_amd import SceneData, synthetic  # noqa: E402
from gasfm_amd.attention import attn_backward_raw, attn_forward_raw  # noqa: E402


def timed(fn, reps, flush):
    ts = []
    for _ in range(reps):
        if flush is not None:
            flush.add_(1.0)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    v = sorted(x.elapsed_time(y) * 1e3 for x, y in ts)
    return v[len(v) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=9)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = synthetic.config4()
    data = SceneData.from_synthetic(sc).to(dev)
    E = sc.num_edges
    H, HC = 4, 32
    g = torch.Generator(device=dev).manual_seed(0)
    XL64 = torch.randn((E, 64), device=dev, generator=g)
    XL32 = {0: XL64[:, :32].contiguous(), 32: XL64[:, 32:].contiguous()}
    att = torch.randn((1, H, HC // H), device=dev, generator=g) * 0.3
    bias = torch.randn(HC, device=dev, generator=g)
    flush = torch.zeros(256 << 20, device=dev)  # 1 GiB
    for name, col, srt in (("proj2scenepoint", 0, True), ("proj2view", 32, False)):
        plan = data.graph_wrappers[name].plan
        N = plan.num_targets
        XR = torch.randn((N, HC), device=dev, generator=g)
        fwd_bytes = E * 4 * HC + 2 * N * 4 * HC + N * 8 * H + (N + 1) * 4
        bwd_bytes = 2 * E * 4 * HC + N * (3 * 4 * HC + 8 * H) + (N + 1) * 4
        for layout, XL in (("interleaved ld64", XL64[:, col:col + HC]), ("contiguous ld32", XL32[col])):
            out, smax, ssum = attn_forward_raw(XL, XR, att, bias, plan, H, 0.2, xl_sorted=srt)
            gout = torch.randn_like(out)
            dXL = torch.empty_like(XL) if XL.is_contiguous() else torch.empty_like(XL64)[:, col:col + HC]
            f = lambda: attn_forward_raw(XL, XR, att, bias, plan, H, 0.2, xl_sorted=srt)  # noqa: E731
            b = lambda: attn_backward_raw(XL, XR, att, bias, plan, H, 0.2, out, smax, ssum, gout,  # noqa: E731
                                          dXL=dXL, xl_sorted=srt)
            r = {"direction": name, "layout": layout}
            for mode, fl in (("cold", flush), ("warm", None)):
                tf, tb = timed(f, args.reps, fl), timed(b, args.reps, fl)
                r[f"fwd_us_{mode}"] = round(tf, 1)
                r[f"fwd_frac_{mode}"] = round(fwd_bytes / tf / 1e3 / 8000, 3)
                r[f"bwd_us_{mode}"] = round(tb, 1)
                r[f"bwd_frac_{mode}"] = round(bwd_bytes / tb / 1e3 / 8000, 3)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
