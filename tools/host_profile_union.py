"""Host-side (Python / ctypes / autograd) cost of one eager training step of the config-3 union batch.

usage: python tools/host_profile_union.py [--steps 10] [--top 45] [--same-thread] [--callers NAME]

Builds one fixed 4-scene union batch the way tools/train_step_bench.py does (device scenes,
10-20 sampled views, rhaug), then runs forward + ESFMLoss + backward eagerly under cProfile and
prints the functions with the largest own time and cumulative time.  The GPU work of this step
replays in ~10 ms (profiles/r3_train_step_capture_floor.txt) while the eager step takes ~29 ms:
the difference is what the host spends per launch.
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
from gasfm_amd import synthetic  # noqa: E402
from gasfm_amd.batch import SceneBatch  # noqa: E402
from gasfm_amd.conf import Conf  # noqa: E402
from gasfm_amd.loss import ESFMLoss  # noqa: E402
from gasfm_amd.scene_device import (apply_rotational_homography_aug_device, sample_data_device,  # noqa: E402
                                    scene_from_dense_device)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--same-thread", action="store_true",
                    help="run the backward on this thread (autograd multithreading off) so cProfile sees it")
    ap.add_argument("--callers", default="", help="also print the callers of functions matching this name")
    args = ap.parse_args()
    if args.same_thread:
        torch.autograd.set_multithreading_enabled(False)
    dev = torch.device("cuda", 0)
    np.random.seed(0)
    torch.manual_seed(0)
    scenes = []
    for i in range(args.batch):
        sc = synthetic.windowed_scene(100, 20_000, seed=100 + i)
        M = torch.from_numpy(sc.dense_M()).to(dev)
        scenes.append(scene_from_dense_device(M, torch.from_numpy(sc.Ns()).to(dev), torch.from_numpy(sc.Ps_gt()).to(dev),
                                              f"train{i}"))
    base = gasfm_amd.learning_conf()
    conf = Conf({"dataset": {"calibrated": True}, "model": base.d["model"],
                 "loss": {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
                          "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True,
                          "hinge_loss_weight": 1.0},
                 "eval": {"calc_reprojerr_with_gtposes_for_depth_pred": False}})
    net = gasfm_amd.GraphAttnSfMNet(conf).to(dev)
    lossf = ESFMLoss(conf)
    datas = [apply_rotational_homography_aug_device(sample_data_device(s, int(np.random.randint(10, 21)), build=False),
                                                    15, 20) for s in scenes]
    union = SceneBatch(datas)

    def step():
        net.zero_grad(set_to_none=True)
        preds = union.split(net(union))
        loss = sum(lossf(p, d) for p, d in zip(preds, datas))
        loss.backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t_plain = (time.perf_counter() - t0) / args.steps
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    print(f"eager step {1e3 * t_plain:.2f} ms (without the profiler), {args.steps} profiled steps follow", flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(args.top)
    st.sort_stats("cumulative").print_stats(args.top)
    if args.callers:
        st.print_callers(args.callers)


if __name__ == "__main__":
    main()
