"""Time the edge-softmax + aggregate kernels alone on the config-4 plans (GPU box).

usage: python tools/attn_bench.py [--reps R] [--points N]
(--points 25000: a rank-of-8 point shard's size, all 1000 cameras; default config 4's 200k)
Prints one JSON line per direction with the forward / backward mean launch time (HIP events
on the launch stream) and the achieved GB/s from the algorithmic byte formulas of
BASELINE.md (forward: E*4*HC + E*4*perm + 2*N*4*HC + N*8*H + (N+1)*4).
GASFM_ATTN_WAVES (read once by libgasfm) overrides the wave cap for sweeps.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gasfm_amd import SceneData, synthetic  # noqa: E402
from gasfm_amd.attention import attn_backward_raw, attn_forward_raw  # noqa: E402


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--points", type=int, default=200_000)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = synthetic.config4(n=args.points)
    data = SceneData.from_synthetic(sc).to(dev)
    E = sc.num_edges
    H, HC = 4, 32
    g = torch.Generator(device=dev).manual_seed(0)
    XL64 = torch.randn((E, 64), device=dev, generator=g)
    att = torch.randn((1, H, HC // H), device=dev, generator=g) * 0.3
    bias = torch.randn(HC, device=dev, generator=g)
    for name, col, srt in (("proj2scenepoint", 0, False), ("proj2scenepoint", 0, True), ("proj2view", 32, False)):
        plan = data.graph_wrappers[name].plan
        N = plan.num_targets
        XL = XL64[:, col:col + HC]
        XR = torch.randn((N, HC), device=dev, generator=g)
        out, smax, ssum = attn_forward_raw(XL, XR, att, bias, plan, H, 0.2, xl_sorted=srt)
        gout = torch.randn_like(out)
        t_f = _time(lambda: attn_forward_raw(XL, XR, att, bias, plan, H, 0.2, xl_sorted=srt), args.reps)
        t_b = _time(lambda: attn_backward_raw(XL, XR, att, bias, plan, H, 0.2, out, smax, ssum, gout,
                                              xl_sorted=srt), args.reps)
        perm = plan.perm is not None and not srt
        fwd_bytes = E * 4 * HC + E * 4 * perm + 2 * N * 4 * HC + N * 8 * H + (N + 1) * 4
        bwd_bytes = 2 * E * 4 * HC + E * 4 * perm + N * (3 * 4 * HC + 8 * H) + (N + 1) * 4
        label = name + (" (XL in segment order)" if srt else "")
        print(json.dumps({"direction": label, "waves": os.environ.get("GASFM_ATTN_WAVES", "default"),
                          "n_items": plan.n_items, "fwd_us": round(t_f, 1),
                          "fwd_GBps": round(fwd_bytes / t_f / 1e3, 1), "bwd_us": round(t_b, 1),
                          "bwd_GBps": round(bwd_bytes / t_b / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
