"""Point-side kernel microbench (GPU box): tail fwd/bwd and hub fwd/bwd_c/bwd_ab/bwd at n = 25k and
200k rows (the per-rank and whole config-4 point counts), mean of 20 launches with HIP events.

usage: [GASFM_LIB=variant.so] python tools/point_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import _native  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    r = lambda *s: torch.randn(*s, device=dev) * 0.1  # noqa: E731
    for N in [int(a) for a in sys.argv[1:]] or (25_000, 200_000):
        prev, agg, dout = r(N, 64), r(N, 32), r(N, 64)
        Wp, bp, g, b, Wm, bm = r(64, 32), r(64), 1 + r(64), r(64), r(64, 64), r(64)
        out, dx, dagg = r(N, 64), r(N, 64), r(N, 32)
        rows, cols = _native.point_tail_part_shape(N, True)
        part = r(rows, cols)
        t_tf = timeit(lambda: _native.point_tail_fwd(prev, agg, Wp, bp, g, b, 1e-5, Wm, bm, out))
        t_tb = timeit(lambda: _native.point_tail_bwd(dout, prev, agg, Wp, bp, g, b, 1e-5, Wm, dx, dagg, part))
        X = r(N, 64)
        gA, bA, WA, WB, bB = 1 + r(64), r(64), r(32, 64), r(64, 64), r(64)
        gC, bC, WC, bWC, WD, bD = 1 + r(64), r(64), r(32, 64), r(32), r(32, 32), r(32)
        SA, XL, XR = r(N, 32), r(N, 64), r(N, 32)
        t_hf = timeit(lambda: _native.point_hub_fwd(X, 1e-5, gA, bA, WA, SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR))
        rc, cc = _native.point_hub_part_shape(N, 1, True)
        ra, ca = _native.point_hub_part_shape(N, 0, True)
        pc, pa = r(rc, cc), r(ra, ca)
        dXR, dSA, dXL, dskip, dp = r(N, 32), r(N, 32), r(N, 64), r(N, 64), r(N, 64)
        t_hc = timeit(lambda: _native.point_hub_bwd_c(X, 1e-5, gC, bC, WC, bWC, WD, dXR, dskip, dp, pc))
        t_ha = timeit(lambda: _native.point_hub_bwd_ab(X, 1e-5, gA, bA, WA, WB, dSA, dXL, dp, dp, pa))
        dp2 = r(N, 64)
        t_h1 = timeit(lambda: _native.point_hub_bwd(X, 1e-5, gA, bA, WA, WB, gC, bC, WC, bWC, WD, dSA, dXL, dXR,
                                                    dskip, dp2, pa, pc))
        print(f"kernel us N={N}: tail_fwd {t_tf:.1f} tail_bwd {t_tb:.1f} hub_fwd {t_hf:.1f} "
              f"hub_bwd_c {t_hc:.1f} hub_bwd_ab {t_ha:.1f} hub_bwd (one pass) {t_h1:.1f} "
              f"(part rows tail {rows}, hub {rc}/{ra})", flush=True)


if __name__ == "__main__":
    main()
