"""CPU baseline (oracle at PyG op granularity, torch CPU fp32, fwd+bwd) at several fractions of the
config-4 workload: is the bench's 10 % sample's edges/s representative of the full scene?

usage: python tools/cpu_baseline_scaling.py [--scales 0.05 0.1 0.25 0.5 1.0] [--reps 1]
Prints one JSON line: per scale (m, n, E, s/step, edges/s), threads, CPU model.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gasfm_amd  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402
from oracle import gasfm_ref, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scales", type=float, nargs="+", default=[0.05, 0.1, 0.25, 0.5, 1.0])
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    threads = bench.host_threads()
    torch.set_num_threads(threads)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf())
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in net.state_dict().items()}
    gasfm_ref.PYG_FAITHFUL = True
    rows = []
    for s in a.scales:
        sc = synthetic.scaled_config4(s, seed=4) if s < 1 else synthetic.config4()
        g = scenes.graph_from_edges(sc.cam, sc.pt, sc.m, sc.n)
        vals = torch.from_numpy(sc.normalized_values())
        ts = []
        for it in range(a.reps + (1 if s < 0.5 else 0)):
            t0 = time.perf_counter()
            out = gasfm_ref.forward(sd, vals, g, dtype=torch.float32)
            (out["Ps_norm"].sum() + out["pts3D"].sum()).backward()
            ts.append(time.perf_counter() - t0)
            for v in sd.values():
                v.grad = None
            del out
        t = float(np.median(ts[-a.reps:]))
        rows.append({"scale": s, "m": sc.m, "n": sc.n, "E": sc.num_edges, "s_per_step": t,
                     "edges_per_s": sc.num_edges / t})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"threads": threads, "cpu": bench.cpu_model(), "torch": torch.__version__, "rows": rows}))


if __name__ == "__main__":
    main()
