"""Multi-scene learning step (BASELINE config 3 shape) with the whole per-sample data path on the device.

usage: python tools/train_step_bench.py [--scenes 12] [--batch 4] [--steps 10] [--host]

Synthetic stand-ins for the 12 Euclidean training scenes (windowed visibility, m = 100 views,
n = 20k points, dense M resident in HBM).  One step follows train.py:60-140 for a batch of
scenes: per scene sample 10-20 consecutive views (SceneData.sample_data), rotational homography
augmentation 15 / 20 degrees (conf rhaug-15-20), graph build, forward, ESFMLoss, the per-step
core errors (compute_core_errors: a host sync per scene, as the reference's .item() calls), then
one backward of the batch loss and an Adam step (--outliers 0.1: config 5's outlier injection, the
model on the injected scene, the loss on the clean one).  The batch's forwards run as ONE forward over the
union of the scene graphs (gasfm_amd/batch.py); --per-scene also times train.py's one forward per
scene.  Every per-sample stage runs on the device
(scene_device.py, loss.py, evaluation.py); --host instead samples on the CPU and builds the graph
with the host builder (no augmentation), the way the reference's DataLoader workers feed the GPU.
Prints one JSON line per mode: scenes/s and the mean ms per stage.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gasfm_amd  # noqa: E402
from gasfm_amd import evaluation, synthetic  # noqa: E402
from gasfm_amd.batch import forward_batch  # noqa: E402
from gasfm_amd.outliers import inject_outliers  # noqa: E402
from gasfm_amd.conf import Conf  # noqa: E402
from gasfm_amd.loss import ESFMLoss  # noqa: E402
from gasfm_amd.scene_device import (apply_rotational_homography_aug_device, sample_data_device,  # noqa: E402
                                    sample_indices, scene_from_dense_device)


def make_scenes(k, m, n, dev):
    out = []
    for i in range(k):
        sc = synthetic.windowed_scene(m, n, seed=100 + i)
        M = torch.from_numpy(sc.dense_M()).to(dev)
        out.append(scene_from_dense_device(M, torch.from_numpy(sc.Ns()).to(dev), torch.from_numpy(sc.Ps_gt()).to(dev),
                                           f"train{i}"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=12)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--views", type=int, default=100)
    ap.add_argument("--points", type=int, default=20_000)
    ap.add_argument("--host", action="store_true", help="also time the host-side data path")
    ap.add_argument("--outliers", type=float, default=0.0,
                    help="outlier injection rate (config 5: rhaug-15-20 + 0.1 outliers), 0 = off")
    ap.add_argument("--per-scene", action="store_true",
                    help="also time one forward per scene (train.py's loop) beside the batched union forward")
    ap.add_argument("--captured", action="store_true",
                    help="also time the captured step (static_batch.StaticTrainer: the batch padded to a bucket, "
                         "forward + loss + errors + backward replayed as one hipGraph per bucket)")
    ap.add_argument("--prime", type=int, default=40,
                    help="--captured: batches run before the timed steps (they create and capture the buckets)")
    ap.add_argument("--pipeline", action="store_true",
                    help="also time the captured step with the next batch prepared on a second stream (prefetch)")
    ap.add_argument("--gasfm-adam", action="store_true",
                    help="--captured: gasfm_amd.optim.Adam (one HIP launch) instead of torch's captured fused Adam")
    ap.add_argument("--no-eager", action="store_true", help="skip the eager union mode (e.g. to profile --captured)")
    ap.add_argument("--progress", type=int, default=10, help="a progress line every this many batches")
    ap.add_argument("--phases", action="store_true",
                    help="--captured: also time the trainer's phases with a synchronize between them (slower)")
    ap.add_argument("--capture-floor", action="store_true",
                    help="also time one FIXED batch's forward + loss + backward captured as a hipGraph and "
                         "replayed (the GPU-side floor of the union step, without the host's launch cost)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
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
    lossf = ESFMLoss(conf)
    # torch's fused Adam (one kernel chain over all 145M parameters; train.py uses Adam's default foreach)
    opt = torch.optim.Adam(net.parameters(), lr=1e-4, fused=True)

    def prep_device(full):
        s = sample_data_device(full, int(np.random.randint(10, 21)), build=False)  # graph built once, after rhaug
        return apply_rotational_homography_aug_device(s, 15, 20)

    def prep_host(full):
        idx = sample_indices(len(full.y), int(np.random.randint(10, 21)), adjacent=True)
        m_idx = np.sort(np.concatenate((2 * idx, 2 * idx + 1)))
        M = full._M.cpu().numpy()[m_idx]
        xs = M.reshape(len(idx), 2, -1)
        keep = ((np.abs(xs).sum(1) != 0).sum(0) >= 2)
        d = gasfm_amd.SceneData(torch.from_numpy(np.ascontiguousarray(M[:, keep])), full.Ns.cpu()[idx],
                                full.y.cpu()[idx], full.scene_name)
        return d.to(dev)

    def run(prep, steps, warmup, batched=True):
        t_prep = t_fb = t_opt = 0.0
        n_done = 0
        repro = []
        for it in range(warmup + steps):
            batch = [scenes[int(i)] for i in np.random.choice(len(scenes), args.batch, replace=False)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            datas = [prep(s) for s in batch]
            # config 5: the model sees the outlier-injected scene, the loss the clean one (train.py:73-90)
            inputs = datas if not args.outliers else [inject_outliers(d, args.outliers, log=lambda s: None)
                                                      for d in datas]
            keep = [k for k, d in enumerate(inputs) if d is not None]
            datas, inputs = [datas[k] for k in keep], [inputs[k] for k in keep]
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            opt.zero_grad()
            batch_loss = 0.0
            preds = forward_batch(net, inputs) if batched else None
            for k, d in enumerate(datas):
                pred = preds[k] if batched else net(inputs[k])
                batch_loss = batch_loss + lossf(pred, d)
                repro.append(evaluation.compute_core_errors(d, pred, conf)["our_repro"])
                if os.environ.get("TSB_DEBUG"):
                    print(it, d.x.shape, int(d.x.pts_per_cam.min()), "pred finite",
                          bool(torch.isfinite(pred["Ps_norm"]).all()), bool(torch.isfinite(pred["pts3D"]).all()),
                          "loss", float(batch_loss), "repro", repro[-1], flush=True)
            batch_loss.backward()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            opt.step()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            if it >= warmup:
                t_prep += t1 - t0
                t_fb += t2 - t1
                t_opt += t3 - t2
                n_done += len(datas)
        tot = t_prep + t_fb + t_opt
        return {"scenes_per_s": n_done / tot, "ms_per_step": 1e3 * tot / steps,
                "ms_data_prep": 1e3 * t_prep / steps, "ms_fwd_bwd_loss_errors": 1e3 * t_fb / steps,
                "ms_adam": 1e3 * t_opt / steps, "first_repro_px": float(repro[0]),
                "last_repro_px": float(repro[-1])}

    def run_pipelined(prep, steps, prime):
        """The captured step with the next batch's data path (sampling, augmentation, scene build,
        outlier injection, batch statistics) prepared on a second stream while this batch replays --
        the reference's DataLoader prefetch, on the device.  Wall time per step."""
        from gasfm_amd.optim import Adam
        from gasfm_amd.static_batch import BatchStats, StaticTrainer
        trainer = StaticTrainer(net, lossf, optimizer=Adam(net.parameters(), lr=1e-4))
        side = torch.cuda.Stream()
        main = torch.cuda.current_stream()

        def prepare(first=False):
            batch = [scenes[int(i)] for i in np.random.choice(len(scenes), args.batch, replace=False)]
            if first:  # the scenes were made on the main stream; later batches read only them (no wait)
                side.wait_stream(main)
            with torch.cuda.stream(side):
                datas = [prep(s) for s in batch]
                inputs = datas if not args.outliers else [inject_outliers(d, args.outliers, log=lambda s: None)
                                                          for d in datas]
                keep = [k for k, d in enumerate(inputs) if d is not None]
                datas, inputs = [datas[k] for k in keep], [inputs[k] for k in keep]
                st = BatchStats(inputs)  # its one host read waits for this stream only
            return datas, inputs, st

        repro = []
        nxt = prepare(first=True)
        t_start = None
        per_step = []  # (wall seconds, captured a new bucket)
        for it in range(prime + steps):
            if it == prime:
                torch.cuda.synchronize()
                t_start = time.perf_counter()
                caps_before = trainer.captures
            if it % args.progress == 0:
                print(f"pipelined: batch {it}/{prime + steps}, buckets {len(trainer.buckets)}", file=sys.stderr,
                      flush=True)
            t0, c0 = time.perf_counter(), trainer.captures
            datas, inputs, st = nxt
            main.wait_stream(side)
            loss, err = trainer.step(datas, inputs, stats=st, read_errors=False)
            nxt = prepare()  # the host prepares the next batch while the GPU replays this one
            repro.extend(trainer.errors(err))  # host sync on this step (the batch tensors stay alive until here)
            if it >= prime:
                per_step.append((time.perf_counter() - t0, trainer.captures != c0))
        torch.cuda.synchronize()
        tot = time.perf_counter() - t_start
        steady = [t for t, cap in per_step if not cap]
        return {"scenes_per_s": steps * args.batch / tot, "ms_per_step": 1e3 * tot / steps,
                "ms_per_step_without_capture_steps": 1e3 * sum(steady) / max(1, len(steady)),
                "scenes_per_s_without_capture_steps": args.batch * len(steady) / max(1e-9, sum(steady)),
                "ms_per_step_median": 1e3 * float(np.median([t for t, _ in per_step])), "prime_batches": prime,
                "buckets": len(trainer.buckets), "captures_in_timed": trainer.captures - caps_before,
                "eager_steps": trainer.eager_steps, "fallbacks": sorted(set(map(str, trainer.fallbacks))),
                "first_repro_px": float(repro[0]), "last_repro_px": float(repro[-1])}

    def run_captured(prep, steps, prime):
        from gasfm_amd.static_batch import StaticTrainer
        # Adam (lr as above): torch's fused Adam with its step captured into each bucket's graph pair
        # (capturable=True), or --gasfm-adam: gasfm_amd.optim.Adam, one launch per step
        if args.gasfm_adam:
            from gasfm_amd.optim import Adam
            copt = Adam(net.parameters(), lr=1e-4)
        else:
            copt = torch.optim.Adam(net.parameters(), lr=1e-4, fused=True, capturable=True)
        trainer = StaticTrainer(net, lossf, optimizer=copt)
        t_prep = t_fb = t_opt = 0.0
        n_done = 0
        repro = []
        caps_before = 0
        t_prime = t_prime_0 = time.perf_counter()
        for it in range(prime + steps):
            if it == prime:
                torch.cuda.synchronize()
                t_prime = time.perf_counter() - t_prime
                caps_before = trainer.captures
                trainer.profile = {} if args.phases else None
            if it % args.progress == 0:
                print(f"captured: batch {it}/{prime + steps}, buckets {len(trainer.buckets)}, captures {trainer.captures}, "
                      f"{time.perf_counter() - t_prime_0:.1f} s", file=sys.stderr, flush=True)
            batch = [scenes[int(i)] for i in np.random.choice(len(scenes), args.batch, replace=False)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            datas = [prep(s) for s in batch]
            inputs = datas if not args.outliers else [inject_outliers(d, args.outliers, log=lambda s: None)
                                                      for d in datas]
            keep = [k for k, d in enumerate(inputs) if d is not None]
            datas, inputs = [datas[k] for k in keep], [inputs[k] for k in keep]
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            copt.zero_grad()
            loss, errs = trainer.step(datas, inputs)  # + Adam; reads the per-scene errors (a host sync)
            repro.extend(errs)
            torch.cuda.synchronize()
            t2 = t3 = time.perf_counter()
            if it >= prime:
                t_prep += t1 - t0
                t_fb += t2 - t1
                t_opt += t3 - t2
                n_done += len(datas)
        tot = t_prep + t_fb + t_opt
        return {"scenes_per_s": n_done / tot, "ms_per_step": 1e3 * tot / steps,
                "ms_data_prep": 1e3 * t_prep / steps, "ms_fill_replay_errors_adam": 1e3 * t_fb / steps,
                "prime_batches": prime, "s_prime": t_prime, "optimizer_graphs": trainer.opt_graphs,
                "buckets": len(trainer.buckets), "captures_in_prime": caps_before,
                "captures_in_timed": trainer.captures - caps_before, "eager_steps": trainer.eager_steps,
                "fallbacks": sorted(set(map(str, trainer.fallbacks))),
                "ms_phases_synced": {k: 1e3 * v / steps for k, v in (trainer.profile or {}).items()},
                "first_repro_px": float(repro[0]),
                "last_repro_px": float(repro[-1])}

    tag = f" + {args.outliers:g} outlier injection" if args.outliers else ""
    if not args.no_eager:
        res = run(prep_device, args.steps, args.warmup)
        print(json.dumps({"mode": "device data path (sample + rhaug" + tag + " + graph build on GPU), batch as one union forward",
                          "batch": args.batch, "scene": f"m={args.views} n={args.points}, 10-20 sampled views", **res}),
              flush=True)
    if args.captured:
        res = run_captured(prep_device, args.steps, args.prime)
        print(json.dumps({"mode": "captured: device data path" + tag + ", the batch padded to a bucket and filled into "
                                  "its static buffers, forward + ESFMLoss + errors + backward replayed as one hipGraph",
                          "batch": args.batch, "scene": f"m={args.views} n={args.points}, 10-20 sampled views", **res}),
              flush=True)
    if args.pipeline:
        res = run_pipelined(prep_device, args.steps, args.prime)
        print(json.dumps({"mode": "captured + pipelined: the next batch's device data path" + tag + " (and its batch "
                                  "statistics) on a second stream while this batch's graph replays; gasfm_amd.optim."
                                  "Adam", "batch": args.batch,
                          "scene": f"m={args.views} n={args.points}, 10-20 sampled views", **res}), flush=True)
    if args.capture_floor:
        from gasfm_amd.batch import SceneBatch
        from gasfm_amd.graph_step import CapturedStep
        batch = [scenes[int(i)] for i in np.random.choice(len(scenes), args.batch, replace=False)]
        datas = [prep_device(s) for s in batch]
        union = SceneBatch(datas)

        def fwd_bwd():
            preds = union.split(net(union))
            loss = sum(lossf(p, d) for p, d in zip(preds, datas))
            loss.backward()
            return loss

        step = CapturedStep(fwd_bwd, net.parameters())
        E = int(union.x.indices.shape[1])
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        t_rep = (time.perf_counter() - t0) / 20
        for _ in range(2):
            opt.zero_grad()
            fwd_bwd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            opt.zero_grad()
            fwd_bwd()
        torch.cuda.synchronize()
        t_eager = (time.perf_counter() - t0) / 5
        print(json.dumps({"mode": "one fixed union batch: forward + ESFMLoss + backward, hipGraph replay vs eager",
                          "batch": args.batch, "edges": E, "captured": step.captured,
                          "fallback": step.fallback_reason, "ms_replay": 1e3 * t_rep, "ms_eager": 1e3 * t_eager}),
              flush=True)
    if args.per_scene:
        res = run(prep_device, args.steps, args.warmup, batched=False)
        print(json.dumps({"mode": "device data path, one forward per scene (train.py's loop)", "batch": args.batch,
                          "scene": f"m={args.views} n={args.points}, 10-20 sampled views", **res}), flush=True)
    if args.host:
        res = run(prep_host, args.steps, args.warmup)
        print(json.dumps({"mode": "host data path (CPU sampling + host graph build, no rhaug, then .to)",
                          "batch": args.batch, "scene": f"m={args.views} n={args.points}", **res}), flush=True)


if __name__ == "__main__":
    main()
