"""Run-to-run / side-stream-vs-not comparison of captured fwd+bwd gradients (debug probe)."""
import sys

import torch

import gasfm_amd
from gasfm_amd import graph_step, streams, synthetic


def main():
    dev = torch.device("cuda:0")
    sc = synthetic.scaled_config4(0.02, seed=7)
    data = gasfm_amd.SceneData.from_synthetic(sc).to(dev)
    torch.manual_seed(0)
    net = gasfm_amd.GraphAttnSfMNet(gasfm_amd.learning_conf(num_layers=4)).to(dev)
    if "--no-defer" in sys.argv:
        net.batch_weight_grads = False
    if "--native-sum" in sys.argv:
        from gasfm_amd import _native, dense
        dense._colsum = lambda a: _native.colsum(a.contiguous())
    gen = torch.Generator().manual_seed(3)
    cP = torch.randn((sc.m, 3, 4), generator=gen).to(dev)
    cX = torch.randn((4, sc.n), generator=gen).to(dev)

    def fwd_bwd():
        pred = net(data)
        loss = (pred["Ps_norm"] * cP).sum() + (pred["pts3D"] * cX).sum()
        loss.backward()
        return loss

    def run(side, capture, reps=1):
        streams.enabled = side
        out = []
        step = graph_step.CapturedStep(fwd_bwd, net.parameters()) if capture else None
        for _ in range(reps):
            if not capture:
                for p in net.parameters():
                    p.grad = None
            loss = step() if capture else fwd_bwd()
            torch.cuda.synchronize()
            out.append((float(loss), {k: p.grad.detach().clone() for k, p in net.named_parameters()}))
        return out

    def cmp(tag, a, b):
        bad = [k for k in a[1] if not torch.equal(a[1][k], b[1][k])]
        md = {k: float((a[1][k] - b[1][k]).abs().max()) for k in bad[:4]}
        print(f"{tag}: loss {a[0]!r} vs {b[0]!r}; {len(bad)} grads differ {md}", flush=True)

    if "--capture-first" in sys.argv:
        c0 = run(False, True, 3)
        c1 = run(True, True, 3)
        cmp("capture off vs on", c0[0], c1[0])
        cmp("capture on r0 vs r2", c1[0], c1[2])
        e0 = run(False, False, 1)
        cmp("capture on vs eager off", c1[0], e0[0])
        cmp("capture off vs eager off", c0[0], e0[0])
        return
    e0 = run(False, False, 2)
    cmp("eager off vs eager off", e0[0], e0[1])
    e1 = run(True, False, 2)
    cmp("eager on vs eager on", e1[0], e1[1])
    cmp("eager off vs eager on", e0[0], e1[0])
    c0 = run(False, True, 3)
    cmp("capture off r0 vs r1", c0[0], c0[1])
    cmp("capture off vs eager off", c0[0], e0[0])
    c1 = run(True, True, 3)
    cmp("capture on r0 vs r1", c1[0], c1[1])
    cmp("capture on r1 vs r2", c1[1], c1[2])
    cmp("capture on vs eager off", c1[0], e0[0])


if __name__ == "__main__":
    main()
