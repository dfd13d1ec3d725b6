"""segment_rowsum on a config-4-sized point plan, output saved for a cross-library bitwise check:
python tools/rowsum_bitwise.py OUT.pt [REF.pt] (with REF: assert torch.equal and print the time)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import _native  # noqa: E402
from gasfm_amd.attention import AttnPlan  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(5)
    n, E = 200_000, 4_000_000
    pt = torch.randint(0, n, (E,), generator=gen)
    pt[:n] = torch.arange(n)  # every point has an edge; a few long segments below
    pt[n:n + 3000] = 7
    plan = AttnPlan.from_targets(pt, n).to(dev)
    X = torch.randn(E, 32, generator=gen).to(dev)
    out = torch.empty(n, 32, device=dev)
    part = torch.empty(max(plan.n_part_rows, 1), 32, device=dev)
    run = lambda: _native.segment_rowsum(plan.items, plan.n_items, plan.perm, X, 0.25, out, part)  # noqa: E731
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        run()
    b.record()
    torch.cuda.synchronize()
    res = torch.cat([out.flatten(), part.flatten()]).cpu()
    torch.save(res, sys.argv[1])
    print(f"segment_rowsum {a.elapsed_time(b) * 1e3 / 20:.1f} us/launch (incl. launch gaps), items {plan.n_items}")
    if len(sys.argv) > 2:
        ref = torch.load(sys.argv[2], weights_only=True)
        assert torch.equal(res, ref), "segment_rowsum outputs differ from the reference library's"
        print("bitwise equal to", sys.argv[2])


if __name__ == "__main__":
    main()
