"""The deferred weight-gradient column sums of one eager config-4 step (gasfm_colsum_multi): number
of jobs, their shapes and the bytes the batched launch reads, to price its time against HBM."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gasfm_amd  # noqa: E402
from gasfm_amd import _native, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    emul = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    sc = synthetic.windowed_scene(1000, 200_000, seed=4)
    torch.manual_seed(0)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=12))
    if emul:
        from gasfm_amd import distributed as gdist
        data = gdist.shard_scene(sc, 0, emul, cameras=True, emulate=True).to(dev)
        model = gdist.ShardedGraphAttnSfMNet(net.to(dev), cameras=True)
    else:
        data = gasfm_amd.SceneData.from_synthetic(sc).to(dev)
        model = net.to(dev)
    seen = []
    orig = _native._flush_param_colsums

    def spy(task, final=True):
        with _native._PENDING_LOCK:
            jobs = list(_native._PENDING.get(task, []))
        seen.append([(j[3], j[4]) for j in jobs])
        return orig(task, final)

    _native._flush_param_colsums = spy
    for _ in range(2):
        pred = model(data)
        loss = pred["Ps_norm"].sum() + pred["pts3D"].sum()
        loss.backward()
        if emul:
            model.sync_grads()
        for p in model.parameters():
            p.grad = None
    torch.cuda.synchronize()
    jobs = seen[-1]
    floats = sum(r * c for r, c in jobs)
    print(f"flushes per step {len(seen) // 2}, jobs {len(jobs)}, partial floats {floats} "
          f"({floats * 4 / 1e6:.1f} MB read), output floats {sum(c for _, c in jobs)}")
    for (r, c), k in Counter(jobs).most_common(20):
        print(f"  {k:3d} x [{r} x {c}] = {k * r * c * 4 / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
