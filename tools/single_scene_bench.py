"""Config 2 as a measured workload: the single-scene optimisation step of
/root/reference/code/single_scene_optimization.py:15-123 (train.py:60-152 with one scene: forward,
ESFMLoss, backward, Adam step) with the 9-block optim conf (confs/gasfm/optim_euc_gasfm.conf:6-17).

The scene is synthetic.config2_standin(): a windowed-visibility stand-in with AlcatrazCourtyard's
size (133 views x 23,674 points, E = 142,104 projections); the dataset is absent offline, so the
shape is the measured quantity, not the data.  Random-init weights of the optim architecture.

Prints one JSON line per mode:
  captured  forward + loss + backward replayed as one hipGraph (graph_step.CapturedStep), then the
            fused Adam step (torch.optim.Adam(fused=True)) -- the production loop;
  eager     the same step launched kernel by kernel from Python/autograd.
usage: python tools/single_scene_bench.py [--steps K] [--warmup W] [--eager-only]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import gasfm_amd  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402
from gasfm_amd.graph_step import CapturedStep  # noqa: E402
from gasfm_amd.loss import ESFMLoss  # noqa: E402

LOSS = {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
        "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True, "hinge_loss_weight": 1.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--eager-only", action="store_true")
    ap.add_argument("--gasfm-adam", action="store_true", help="gasfm_amd.optim.Adam instead of torch's fused Adam")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    sc = synthetic.config2_standin()
    conf = gasfm_amd.optim_conf()
    conf.put("loss", dict(LOSS))
    net = gasfm_amd.GraphAttnSfMNet(conf).to(dev)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(dev)
    lossf = ESFMLoss(conf)
    if args.gasfm_adam:  # gasfm_amd.optim.Adam: torch.optim.Adam's update in one HIP launch
        from gasfm_amd.optim import Adam
        opt = Adam(net.parameters(), lr=1e-4)
    else:
        opt = torch.optim.Adam(net.parameters(), lr=1e-4, fused=True)
    adam_name = "one-launch Adam (gasfm_amd.optim)" if args.gasfm_adam else "fused Adam step"

    def fwd_bwd():
        loss = lossf(net(data), data)
        loss.backward()
        return loss

    modes = ["eager"] if args.eager_only else ["captured", "eager"]
    for mode in modes:
        if mode == "captured":
            step_fn = CapturedStep(fwd_bwd, net.parameters(), warmup=args.warmup)
            execution = (f"hipGraph replay of forward+loss+backward, {adam_name}" if step_fn.captured
                         else f"eager fallback ({step_fn.fallback_reason})")
        else:
            def step_fn():
                for p in net.parameters():
                    p.grad = None
                return fwd_bwd()
            for _ in range(args.warmup):
                step_fn()
                opt.step()
            execution = f"eager forward+loss+backward (one launch per kernel), {adam_name}"
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step_fn()
            opt.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        print(json.dumps({
            "metric": "config-2 single-scene optimisation steps/s (fwd + ESFMLoss + bwd + Adam)",
            "mode": mode, "execution": execution, "ms_per_step": dt * 1e3, "steps_per_s": 1.0 / dt,
            "edges_per_s": sc.num_edges / dt, "loss": float(loss.detach()), "steps": args.steps,
            "warmup": args.warmup, "dtype": "fp32",
            "config": {"workload": "config 2 stand-in (synthetic.config2_standin, AlcatrazCourtyard size)",
                       "cameras": sc.m, "points": sc.n, "edges": sc.num_edges, "blocks": 9,
                       "conf": "optim_euc_gasfm (9 blocks, full widths)"},
            "data": "synthetic windowed visibility; random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
