"""Config-5 training step, point-sharded (gasfm_amd/dist_train.py): one sampled + augmented +
outlier-injected scene per step (the GASFM confs' batch_size = 1), identical on every rank.

    python tools/dist_train_bench.py --emulate-world 8      # rank 0's share of an 8-GPU step, 1 GPU
    torchrun --nproc-per-node N tools/dist_train_bench.py   # N ranks over RCCL

Synthetic stand-ins for the 12 Euclidean training scenes (m = 100 views, n = 20k points, dense M
resident in HBM) as tools/train_step_bench.py.  Per step: seeded draws (the same on every rank),
sampling + rhaug 15/20 + 10 % outliers on the device, the shard (plans on the host), forward,
ESFMLoss, compute_core_errors, backward, sync_grads, gasfm Adam.  Prints one JSON line: ms per
step split into the data path and the sharded step, edges per step.  --emulate-world replaces
every collective by a local copy (timing only, numerically meaningless).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=12)
    ap.add_argument("--views", type=int, default=100)
    ap.add_argument("--points", type=int, default=20_000)
    ap.add_argument("--outliers", type=float, default=0.1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--emulate-world", type=int, default=0)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", 1))
    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=dev)

    import gasfm_amd
    from gasfm_amd.conf import Conf
    from gasfm_amd.dist_train import ShardedTrainer, sample_training_scene
    from gasfm_amd.loss import ESFMLoss
    from gasfm_amd.optim import Adam
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from train_step_bench import make_scenes

    np.random.seed(0)
    torch.manual_seed(0)
    scenes = make_scenes(args.scenes, args.views, args.points, dev)
    base = gasfm_amd.learning_conf()
    conf = Conf({"dataset": {"calibrated": True}, "model": base.d["model"],
                 "loss": {"infinity_pts_margin": 1e-4, "pts_grad_equalization_pre_perspective_divide": True,
                          "normalize_grad_wrt_valid_projections_only": True, "hinge_loss": True,
                          "hinge_loss_weight": 1.0},
                 "eval": {"calc_reprojerr_with_gtposes_for_depth_pred": False}})
    net = gasfm_amd.GraphAttnSfMNet(conf).to(dev)
    trainer = ShardedTrainer(net, ESFMLoss(conf), optimizer=Adam(net.parameters(), lr=1e-4),
                             emulate_world=args.emulate_world if world == 1 else 0)
    t_prep = t_step = 0.0
    edges = []
    errs = []
    for it in range(args.warmup + args.steps):
        np.random.seed(1000 + it)  # the same draws on every rank
        torch.manual_seed(1000 + it)
        full = scenes[int(np.random.randint(len(scenes)))]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d, inp = sample_training_scene(full, args.outliers)
        if inp is None:
            continue
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        loss, err = trainer.step(d, inp)
        errs.append(float(err))  # compute_core_errors' host read (train.py:91)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if it >= args.warmup:
            t_prep += t1 - t0
            t_step += t2 - t1
            edges.append(int(d.x.indices.shape[1]))
    n = len(edges)
    if rank == 0:
        W = args.emulate_world if world == 1 and args.emulate_world > 1 else world
        print(json.dumps({
            "mode": ("emulated rank 0 of %d (collectives replaced by local copies: per-rank compute only)" % W
                     if world == 1 and args.emulate_world > 1 else f"{world} ranks (RCCL)"),
            "step": "config 5: sample 10-20 views + rhaug 15/20 + %g outliers (device), point shard (host plans), "
                    "sharded forward + ESFMLoss + core errors + backward + sync_grads + gasfm Adam, eager" % args.outliers,
            "scenes": f"{args.scenes} synthetic m={args.views} n={args.points}", "steps": n,
            "ms_per_step": 1e3 * (t_prep + t_step) / n, "ms_data_prep": 1e3 * t_prep / n,
            "ms_sharded_step": 1e3 * t_step / n, "mean_edges_per_scene": float(np.mean(edges)),
            "first_repro_px": errs[0], "last_repro_px": errs[-1]}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
