"""torch.profiler view of one eager step (op names + input shapes + device time), GPU box.

usage: python tools/torch_prof.py [--n N] [--emulate-world W] [--stacks]
"""
import argparse
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gasfm_amd  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=25_000)
    ap.add_argument("--rows", type=int, default=40)
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="rank 0 of a W-way points + cameras shard (bench.py --emulate-world)")
    ap.add_argument("--stacks", action="store_true",
                    help="also list the Python call sites of the aten ops that launch device work")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = synthetic.windowed_scene(1000, args.n, seed=4)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf()).to(dev)
    cP = torch.randn((sc.m, 3, 4), device=dev)
    cX = torch.randn((4, sc.n), device=dev)
    if args.emulate_world > 1:
        from gasfm_amd import distributed as gdist
        data = gdist.shard_scene(sc, 0, args.emulate_world, cameras=True, emulate=True).to(dev)
        model = gdist.ShardedGraphAttnSfMNet(net, cameras=True)
        cX = cX[:, data.point_slice].contiguous()
    else:
        data = gasfm_amd.SceneData.from_synthetic(sc).to(dev)
        model = net

    def step():
        p = model(data)
        ((p["Ps_norm"] * cP).sum() + (p["pts3D"] * cX).sum()).backward()
        if args.emulate_world > 1:
            model.sync_grads()
        for q in net.parameters():
            q.grad = None
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=args.stacks) as prof:
        step()
        torch.cuda.synchronize()
    ev = [e for e in prof.key_averages(group_by_input_shape=True) if e.self_device_time_total > 0]
    ev.sort(key=lambda e: -e.self_device_time_total)
    tot = sum(e.self_device_time_total for e in ev)
    print(f"self device time total {tot / 1e3:.2f} ms")
    for e in ev[:args.rows]:
        print(f"{e.self_device_time_total / 1e3:7.3f} ms {e.count:5d}x  {e.key[:60]:60s} {str(e.input_shapes)[:90]}")
    # aten ops that launch device work, by launch count (the per-launch floor dominates small ops)
    ops = [e for e in prof.key_averages(group_by_input_shape=True)
           if e.key.startswith("aten::") and e.device_time_total > 0]
    ops.sort(key=lambda e: -e.count)
    print("\naten ops by count (with device time):")
    for e in ops[:args.rows]:
        print(f"{e.count:5d}x {e.device_time_total / 1e3:7.3f} ms  {e.key[:40]:40s} {str(e.input_shapes)[:100]}")
    if args.stacks:
        # gasfm_amd call sites of aten ops with device work (excluding the libgasfm launches)
        print("\naten ops with device work by gasfm_amd call site:")
        from collections import defaultdict
        agg = defaultdict(lambda: [0, 0.0])
        for e in prof.events():
            if not e.name.startswith("aten::") or e.device_time_total <= 0:
                continue
            st = [f for f in (e.stack or []) if "gasfm_amd" in f][:2]
            key = (e.name, " <- ".join(st) if st else "(no gasfm_amd frame)")
            agg[key][0] += 1
            agg[key][1] += e.device_time_total
        for (name, site), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:args.rows]:
            print(f"{n:5d}x {t / 1e3:7.3f} ms  {name[:28]:28s} {site[:200]}")


if __name__ == "__main__":
    main()
