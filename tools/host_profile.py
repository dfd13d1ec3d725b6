"""Host-side (Python) cost of one config-3-shaped training step: cProfile of forward + ESFMLoss +
core errors + backward for a batch of sampled scenes (the eager path, GPU work is tiny).

usage: python tools/host_profile.py [--batch 4] [--steps 3] [--top 45]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gasfm_amd  # noqa: E402
from gasfm_amd import evaluation, synthetic  # noqa: E402
from gasfm_amd.conf import Conf  # noqa: E402
from gasfm_amd.loss import ESFMLoss  # noqa: E402
from gasfm_amd.scene_device import (apply_rotational_homography_aug_device, sample_data_device,  # noqa: E402
                                    scene_from_dense_device)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--per-scene", action="store_true", help="one forward per scene (default: the union batch)")
    ap.add_argument("--prep", action="store_true", help="profile the device data path instead (sample + rhaug + "
                                                        "0.1 outlier injection)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    np.random.seed(0)
    torch.manual_seed(0)
    scenes = []
    for i in range(4):
        sc = synthetic.windowed_scene(100, 20000, seed=100 + i)
        scenes.append(scene_from_dense_device(torch.from_numpy(sc.dense_M()).to(dev), torch.from_numpy(sc.Ns()).to(dev),
                                              torch.from_numpy(sc.Ps_gt()).to(dev), f"train{i}"))
    base = gasfm_amd.learning_conf()
    conf = Conf({"dataset": {"calibrated": True}, "model": base.d["model"],
                 "loss": {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
                          "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True,
                          "hinge_loss_weight": 1.0},
                 "eval": {"calc_reprojerr_with_gtposes_for_depth_pred": False}})
    net = gasfm_amd.GraphAttnSfMNet(conf).to(dev)
    lossf = ESFMLoss(conf)

    from gasfm_amd.batch import forward_batch
    from gasfm_amd.outliers import inject_outliers

    def prep():
        return [apply_rotational_homography_aug_device(sample_data_device(s, int(np.random.randint(10, 21))), 15, 20)
                for s in scenes[:args.batch]]

    def step():
        if args.prep:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            datas = [inject_outliers(d, 0.1, log=lambda s: None) for d in prep()]
            torch.cuda.synchronize()
            return time.perf_counter() - t0
        datas = prep()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        net.zero_grad()
        tot = 0.0
        preds = None if args.per_scene else forward_batch(net, datas)
        for k, d in enumerate(datas):
            pred = net(d) if args.per_scene else preds[k]
            tot = tot + lossf(pred, d)
            evaluation.compute_core_errors(d, pred, conf)
        tot.backward()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for _ in range(2):
        step()
    pr = cProfile.Profile()
    ts = []
    for _ in range(args.steps):
        pr.enable()
        ts.append(step())
        pr.disable()
    print("data prep" if args.prep else "fwd+loss+errors+bwd", "ms per step:", [round(1e3 * t, 1) for t in ts])
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(args.top)
    st.sort_stats("cumulative").print_stats(args.top)


if __name__ == "__main__":
    main()
