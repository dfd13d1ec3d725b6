"""GAT-stack edges/sec (fwd+bwd) on the synthetic 1k-camera / 200k-point scene (BASELINE config 4).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

A step = one forward + backward of the full GraphAttnSfMNet (12 blocks, learning
conf widths, fp32) over the whole scene, loss = a fixed linear functional of
Ps_norm and pts3D.  Inputs (scene graph, features, weights)
are resident in HBM before timing.  value = E * K / (max over ranks of the
timed wall time).  With N > 1 the scene's points are sharded over the ranks
(gasfm_amd.distributed) — strong scaling: the scene is fixed.

Also reported, on the same line:
  roofline      the step's dominant kernel: the fused camera-attention + edge-prologue
                backward (edge_cam_pbwd_kernel<LN,RES>, ~23 % of the step), timed live with
                HIP events around each of its launches on its stream right after the timed
                region.  Its MFMA floor (12,288 fp32 FLOP per edge at 157.3 TF/s) is above its
                HBM floor (512 B per edge at 8 TB/s), so achieved = FLOP / mean duration
                against the fp32 MFMA peak; the HBM rate is reported beside it.
  roofline_attention  the fused edge-softmax + aggregation forward of the point direction
                (attn_fwd_grp_kernel<4,1>, the north-star GATv2 kernel), timed the same way;
                achieved = SURVEY §8(d)'s algorithmic bytes / mean duration; peak 8.0 TB/s.
  cpu_baseline  the oracle's torch-CPU restatement of the reference + PyG op sequence
                (oracle.gasfm_ref with PYG_FAITHFUL) on a bounded sample scene,
                rank 0 at N=1 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_F32_PEAK_TFS = 157.3  # dense fp32 MFMA (v_mfma_f32_16x16x4_f32): 64 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz
PBWD_FLOP_PER_EDGE = 12288  # XLc recompute 2,048 + dP_hat (3 products, K = 32) 6,144 + dW (64 x 32) 4,096
PBWD_BYTES_PER_EDGE = 512  # P, dXL point half, dRes read, dP written (camera rows once: + 160 B per camera)
# with the edge epilogue's backward folded in (edge_block.EPI_FOLD, edge_cam_pbwd<.., EPI, DWP>): + dWp
# (32 x 34: 2,176) + dP0 (2 x 32 dots: 128) FLOP, + P0 read 8 + dP0 written 8 bytes per edge
PBWD_FOLD_FLOP_PER_EDGE = PBWD_FLOP_PER_EDGE + 2176 + 128
PBWD_FOLD_BYTES_PER_EDGE = PBWD_BYTES_PER_EDGE + 16
_PROFILES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
# the newest committed per-kernel PMC table (tools/pmc_kernels.sh)
PMC_KERNELS = next((os.path.join(_PROFILES, f) for f in ("r6_pmc_kernels.txt", "r5_pmc_kernels.txt", "r4_pmc_kernels.txt",
                                                          "r3_pmc_kernels.txt")
                    if os.path.exists(os.path.join(_PROFILES, f))), os.path.join(_PROFILES, "r3_pmc_kernels.txt"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


PMC_TRAFFIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r2_pmc_attn_fwd.json")


def pmc_traffic(E, N):
    """HBM bytes per point-direction launch from the committed PMC pass (tools/pmc_traffic.sh:
    2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction), when it was taken on this workload."""
    try:
        with open(PMC_TRAFFIC) as f:
            r = json.load(f)
    except (OSError, ValueError):
        return None
    w = r.get("workload", {})
    if w.get("edges") != E or w.get("points") != N:
        return None
    return r["point"]["traffic_bytes"]


def pmc_kernel_traffic(names, E):
    """HBM bytes per launch of the first of ``names`` in the committed per-kernel PMC table
    (tools/pmc_kernels.sh on this bench: 2 x FETCH_SIZE + WRITE_SIZE), when it was taken on the
    config-4 workload."""
    if E != 4001638:
        return None
    try:
        with open(PMC_KERNELS) as f:
            lines = f.readlines()
        for name in ((names,) if isinstance(names, str) else names):
            key = name.rstrip(">")  # the table truncates names (and round 4 added a template argument)
            for line in lines:
                if line.startswith(key):
                    return float(line.split()[-3]) * 1e6  # total MB column
    except (OSError, ValueError, IndexError):
        return None
    return None


# spin-kernel length (torch.cuda._sleep cycles) issued before each timed launch: the start event, the
# launch and the end event are then all enqueued while the GPU spins, so the events bracket the
# kernel's execution and not the host's enqueue latency (rocprof's in-step durations agree)
HOLD_CYCLES = 2_000_000


class LaunchTimer:
    """HIP events around every call of a gasfm_amd._native launcher (module attribute swapped in place,
    restored by close()) whose arguments ``select`` accepts, on the stream the launch goes to; the
    stream is held by a spin kernel (HOLD_CYCLES) while the three are enqueued."""

    def __init__(self, name, select):
        from gasfm_amd import _native
        self.mod, self.name, self.orig = _native, name, getattr(_native, name)
        self.events = []

        def wrapped(*a, **k):
            if not select(*a, **k):
                return self.orig(*a, **k)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            torch.cuda._sleep(HOLD_CYCLES)
            ev[0].record()
            r = self.orig(*a, **k)
            ev[1].record()
            self.events.append(ev)
            return r
        setattr(_native, name, wrapped)

    def close(self):
        setattr(self.mod, self.name, self.orig)
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.events) / len(self.events) if self.events else None


def attn_fwd_bytes(E, N, H, HC, perm):
    """BASELINE.md algorithmic bytes of one fused edge-softmax + aggregation forward."""
    return E * 4 * HC + E * 4 * int(perm) + N * 4 * HC + N * 4 * HC + N * 8 * H + (N + 1) * 4


def host_threads():
    """Every core this process may run on (sched affinity), capped only by an OMP_NUM_THREADS the
    host sets for its share of the machine (the GPU boxes export 16 per GPU)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# The CPU port's cost is linear in the edge count: its time per step is E-sized tensor ops
# (gathers, index_add, [E, 64] GEMMs) plus camera-sized ops that also shrink with the sample
# (m = 1000 x scale cameras).  tools/cpu_baseline_scaling.py measured edges/s at scales
# 0.05 .. 1.0 (profiles/r2_cpu_baseline_scaling.json): the full config-4 workload runs within
# 16 % of the 10 % sample's edges/s (51.3k vs 59.4k edges/s, 78 s per full step on 16 EPYC 9575F
# threads), so the bench times the sample (a ~16 % optimistic CPU number) and reports its edges/s.
def cpu_baseline(sample_scale, threads, reps=4):
    """Oracle (reference + PyG op sequence, torch CPU fp32) fwd+bwd edges/s on a sample scene."""
    import gasfm_amd
    from gasfm_amd import synthetic
    from oracle import gasfm_ref, scenes
    torch.set_num_threads(threads)
    sc = synthetic.scaled_config4(sample_scale, seed=4)
    g = scenes.graph_from_edges(sc.cam, sc.pt, sc.m, sc.n)
    vals = torch.from_numpy(sc.normalized_values())
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf())
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in net.state_dict().items()}
    gasfm_ref.PYG_FAITHFUL = True
    times = []
    for it in range(1 + reps):  # 1 warm-up + median of reps
        t0 = time.perf_counter()
        out = gasfm_ref.forward(sd, vals, g, dtype=torch.float32)
        (out["Ps_norm"].sum() + out["pts3D"].sum()).backward()
        times.append(time.perf_counter() - t0)
        for v in sd.values():
            v.grad = None
    gasfm_ref.PYG_FAITHFUL = False
    t = float(np.median(times[1:]))
    lo, hi = sc.num_edges / max(times[1:]), sc.num_edges / min(times[1:])
    return {"value": sc.num_edges / t, "unit": "edges/s", "cores": threads, "kind": "port",
            "range": [lo, hi],
            "sample": f"scaled config 4 (m={sc.m}, n={sc.n}, E={sc.num_edges}), 12 blocks, fp32, fwd+bwd, "
                      f"median of {reps} after 1 warm-up ({lo / 1e3:.1f}k-{hi / 1e3:.1f}k edges/s over the {reps}), "
                      f"{t:.2f} s/step, "
                      f"torch {torch.__version__} CPU threads={threads} on {cpu_model()}; edges/s of the sample "
                      f"stands for config 4 (linear in E: profiles/r2_cpu_baseline_scaling.json)"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launcher_argv(gpus, argv, port):
    """The torchrun command that starts ``gpus`` ranks of this bench on one node (one process per
    GPU, RCCL), with the caller's own arguments passed through unchanged."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(gpus, argv, run=None):
    """``bench.py --gpus N`` (N > 1) started without a launcher: run torchrun with N ranks as a CHILD
    process (never exec: nothing here has touched the GPU yet, and the ranks initialise it
    themselves), its stdout / stderr inherited, and return its exit code."""
    import subprocess
    run = run or subprocess.call
    return run(rank_launcher_argv(gpus, argv, _free_port()))


def world_from_env(gpus):
    """(rank, world, local_rank) from the launcher's environment.  Under a launcher, --gpus must
    equal WORLD_SIZE: a mismatch is an error (exit 2), never a silent 1-GPU run."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != gpus:
        log(f"error: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        sys.exit(2)
    return rank, world, local_rank


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    # --cameras / --points: spellings torchrun's own parser does not take for abbreviations
    ap.add_argument("--m", "--cameras", dest="m", type=int, default=1000)
    ap.add_argument("--n", "--points", dest="n", type=int, default=200_000)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="launch every kernel from Python (no hipGraph)")
    ap.add_argument("--cpu-sample-scale", type=float, default=0.1)
    ap.add_argument("--proj-precision", choices=("fp32", "bf16"), default="fp32",
                    help="bf16: the camera-side 1024x1024 projections on the bf16 MFMA kernel (BASELINE config 5)")
    ap.add_argument("--dist", action="store_true",
                    help="run the point-sharded RCCL path even at one rank (under torchrun --nproc-per-node 1)")
    ap.add_argument("--no-cam-shard", action="store_true",
                    help="N > 1: shard the points only (the view chain replicated on every rank)")
    ap.add_argument("--cam-shard-1", action="store_true",
                    help="with --dist at one rank: run the camera-sharded code path anyway (RCCL capture test)")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend at N > 1: nccl (= RCCL, the measured path); gloo stages the "
                         "collectives through the host (a functional test of the N-rank launch, not a measurement)")
    ap.add_argument("--one-gpu", action="store_true",
                    help="with --backend gloo: every rank on cuda:0 (tests the N-rank path on a one-GPU box)")
    ap.add_argument("--emulate-world", type=int, default=0, metavar="W",
                    help="per-rank proxy: rank 0's shard of a W-GPU step on this one GPU, collectives replaced by "
                         "local copies (timing of the per-rank compute; numerically meaningless)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank, world, local_rank = world_from_env(args.gpus)
    if args.one_gpu and args.backend != "gloo":
        log("error: --one-gpu needs --backend gloo (RCCL does not run two ranks on one GPU)")
        sys.exit(2)
    local_rank = 0 if args.one_gpu else local_rank
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist_on = world > 1 or args.dist
    emul = args.emulate_world > 1 and not dist_on
    cams = not args.no_cam_shard
    if dist_on:
        if args.backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group("gloo")
        if torch.distributed.get_world_size() != world:  # n_gpus is the rank count RCCL reports
            log(f"error: RCCL reports {torch.distributed.get_world_size()} ranks, WORLD_SIZE {world}")
            sys.exit(2)
        log(f"[rank {rank}] process group up (world {world})")

    import gasfm_amd
    from gasfm_amd import attention, synthetic

    t0 = time.time()
    sc = synthetic.windowed_scene(args.m, args.n, seed=4)
    E = sc.num_edges
    conf = gasfm_amd.learning_conf(num_layers=args.layers)
    torch.manual_seed(0)
    net = gasfm_amd.GraphAttnSfMNet(conf).set_projection_precision(args.proj_precision)
    if dist_on or emul:
        from gasfm_amd import distributed as gdist
        if emul:
            data = gdist.shard_scene(sc, 0, args.emulate_world, cameras=cams, emulate=True).to(dev)
        else:
            data = gdist.shard_scene(sc, rank, world, cameras=cams and (world > 1 or args.cam_shard_1)).to(dev)
        model = gdist.ShardedGraphAttnSfMNet(net.to(dev), cameras=data.shard.cams is not None)
    else:
        data = gasfm_amd.SceneData.from_synthetic(sc).to(dev)
        model = net.to(dev)
    gen = torch.Generator().manual_seed(123)
    cP = torch.randn((sc.m, 3, 4), generator=gen).to(dev)
    cX = torch.randn((4, sc.n), generator=gen).to(dev)
    log(f"[rank {rank}] scene m={sc.m} n={sc.n} E={E} built+moved in {time.time() - t0:.1f}s")

    cx = cX if not (dist_on or emul) else cX[:, data.point_slice].contiguous()

    def fwd_bwd():
        pred = model(data)
        # replicated outputs enter every rank's loss in full, local points once (distributed.py)
        loss = (pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cx).sum()
        loss.backward()
        if dist_on or emul:
            model.sync_grads()
        return loss

    from gasfm_amd.graph_step import CapturedStep
    if args.eager:
        for _ in range(args.warmup):
            fwd_bwd()
            for p in model.parameters():
                p.grad = None

        def step():
            fwd_bwd()
            for p in model.parameters():
                p.grad = None
        execution = "eager (one Python/autograd launch per kernel)"
    else:
        # warm-up steps run inside CapturedStep (before capture); every timed step replays
        # the captured forward+backward (+ gradient all-reduce) as one hipGraph launch
        agree = None
        if dist_on:
            def agree(ok):  # AND over ranks, one collective outside the graph
                t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if args.backend == "nccl" else "cpu")
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
                return bool(t.item())
        captured = CapturedStep(fwd_bwd, model.parameters(), warmup=args.warmup, agree=agree)
        step = captured
        execution = ("hipGraph replay of the captured forward+backward step" if captured.captured
                     else f"eager fallback ({captured.fallback_reason})")
        log(f"[rank {rank}] {execution}")
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist_on:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([dt], device=dev if args.backend == "nccl" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    # roofline kernel: the point-direction attention forward, in eager steps right after the
    # timed region (events cannot be read out of a replayed graph): events around each of its
    # launches (mean_us: matches rocprof's in-step durations), plus 20 back-to-back re-launches
    # on the inputs of its last launch (mean_us_back_to_back: cache-warm, informational)
    timer = attention.KernelTimer(lambda tag, HC: tag == "proj2scenepoint" and HC == 32, hold_cycles=HOLD_CYCLES)
    attention.KERNEL_TIMER = timer
    timer.enabled = True
    # the dominant kernel: edge_cam_pbwd with LayerNorm and the residual term (blocks 1..11); with the
    # epilogue fold, its launches that carry both epilogue parts (blocks 2..11)
    from gasfm_amd import edge_block
    fold = edge_block.EPI_FOLD
    pbwd = LaunchTimer("edge_cam_pbwd", lambda *a, **k: a[1] is not None and a[7] is not None
                       and (not fold or (k.get("epi") is not None and k.get("dwp") is not None)))
    flop_e = PBWD_FOLD_FLOP_PER_EDGE if fold else PBWD_FLOP_PER_EDGE
    bytes_e = PBWD_FOLD_BYTES_PER_EDGE if fold else PBWD_BYTES_PER_EDGE
    # (round 4: the EPI template argument is an int -- 1 the 32-wide fold, 2 block 0's -- so newer
    # tables print it as a number)
    pbwd_name = (("edge_cam_pbwd_kernel<true, true, 1, true>", "edge_cam_pbwd_kernel<true, true, true, true>") if fold
                 else ("edge_cam_pbwd_kernel<true, true, 0, false>", "edge_cam_pbwd_kernel<true, true, false, false>"))
    for _ in range(2):
        fwd_bwd()
    timer.enabled = False
    attention.KERNEL_TIMER = None
    pbwd_ms = pbwd.close()
    pbwd_launches = len(pbwd.events)
    e_cam = data.graph_wrappers["proj2view"].plan.num_edges
    pbwd_tfs = flop_e * e_cam / (pbwd_ms * 1e-3) / 1e12 if pbwd_ms else None
    pbwd_gbs = bytes_e * e_cam / (pbwd_ms * 1e-3) / 1e9 if pbwd_ms else None
    pbwd_traffic = pmc_kernel_traffic(pbwd_name, e_cam)
    kern_ms = timer.mean_ms()
    b2b_ms = timer.replay_ms(20)
    plan = data.graph_wrappers["proj2scenepoint"].plan
    e_local = plan.num_edges
    n_local = plan.num_targets
    bytes_per_launch = attn_fwd_bytes(e_local, n_local, 4, 32, bool(timer.gathered))
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9 if kern_ms else None

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_sample_scale, host_threads())
        res = {
            "metric": "GAT-stack edges/sec (fwd+bwd) on cam/point scene graph; 1/2/4/8 MI355X",
            "value": E * args.steps / dt,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * dt / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32" if args.proj_precision == "fp32" else "bf16-proj",
            "data": "synthetic (config 4 generator: SfM-like windowed visibility, default_rng(4)); random-init "
                    "weights of the learning_euc GASFM architecture",
            "config": {"workload": f"config 4: m={sc.m} cameras, n={sc.n} points, E={E} projections, "
                                   f"{args.layers}-block GraphAttnSfMNet (learning_euc widths) fwd+bwd"
                                   + ("" if args.proj_precision == "fp32" else
                                      ", camera-side 1024x1024 projections in bf16 on MFMA (fp32 accumulate)"),
                       "cameras": sc.m, "points": sc.n, "edges": E, "blocks": args.layers,
                       "parallelism": (f"emulated rank 0 of {args.emulate_world} ({'points + cameras' if cams else 'points'}"
                                       " sharded; collectives replaced by local copies: per-rank compute only)"
                                       if emul else
                                       f"{'point+camera' if data.shard.cams is not None else 'point'}-sharded x{world}"
                                       + ("" if args.backend == "nccl" else
                                          " (gloo on one GPU: a functional test of the N-rank path, not a measurement)")
                                       if dist_on else "single GPU")},
            "roofline": {"kernel": pbwd_name[0] + ": camera-attention + edge-prologue backward"
                                   + (" + the edge epilogue's backward (dSv, dP0 of the previous block, dWp of this "
                                      "one)" if fold else "") + " (the step's largest kernel), per launch",
                         "bound": "mfma", "achieved": pbwd_tfs, "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": (pbwd_tfs / MFMA_F32_PEAK_TFS) if pbwd_tfs else None,
                         "traffic": pbwd_traffic,
                         "traffic_source": f"profiles/{os.path.basename(PMC_KERNELS)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                           "passes of this bench, per launch"
                                           + (f"; {pbwd_traffic / (bytes_e * e_cam):.2f}x the algorithmic bytes)"
                                              if pbwd_traffic else "; not taken on this workload)"),
                         "flop_per_launch": flop_e * e_cam,
                         "algorithmic_bytes": bytes_e * e_cam,
                         "hbm_achieved_GBps": pbwd_gbs,
                         "hbm_frac": (pbwd_gbs / HBM_PEAK_GBS) if pbwd_gbs else None,
                         "mean_us": pbwd_ms * 1e3 if pbwd_ms else None, "launches_timed": pbwd_launches,
                         "timing": "HIP events on the launch stream around each of its launches in 2 eager steps "
                                   "after the timed region, the stream held by a spin kernel while the events and "
                                   "the launch are enqueued (the host's enqueue latency is not timed; agrees with "
                                   "the rocprof durations inside the replayed step)"},
            "roofline_attention": {"kernel": "attn_fwd_grp_kernel<4,1> point direction (proj2scenepoint), per launch",
                         "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": pmc_traffic(e_local, n_local),
                         "traffic_source": "profiles/r2_pmc_attn_fwd.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                           "passes of this bench, per launch)",
                         "algorithmic_bytes": bytes_per_launch, "mean_us": kern_ms * 1e3 if kern_ms else None,
                         "mean_us_back_to_back": b2b_ms * 1e3 if b2b_ms else None,
                         "launches_timed": len(timer.events),
                         "timing": "HIP events on the launch stream around each of its launches in 2 eager steps "
                                   "after the timed region, the stream held by a spin kernel while the events and "
                                   "the launch are enqueued (mean_us; agrees with the rocprof durations inside the "
                                   "replayed step); mean_us_back_to_back: 20 re-launches on the inputs of its last "
                                   "launch between two events (cache-warm, not used for achieved)"},
            "execution": execution,
            "cpu_baseline": cpu,
        }
        print(json.dumps(res), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
