"""gasfm_gemm_f32 and gasfm_gemm_f32_smallm vs torch (hipBLASLt) on the camera-side shapes: y = x W^T, dx = dy W, dW = dy^T x
at m = 1000 and m = 125 (HIP events, 50 back-to-back launches each)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import _native  # noqa: E402


def t(fn, reps=50):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    dev = torch.device("cuda")
    D = 1024
    W = torch.randn(D, D, device=dev)
    for m in (1000, 125):
        x = torch.randn(m, D, device=dev)
        dy = torch.randn(m, D, device=dev)
        fl = 2 * m * D * D
        for name, hip, ref, sm in (
                ("fwd  x W^T", lambda: _native.gemm_f32(x, W.t()), lambda: x @ W.t(),
                 lambda: _native.gemm_f32_smallm(x, W.t())),
                ("dgrad dy W", lambda: _native.gemm_f32(dy, W), lambda: dy @ W, lambda: _native.gemm_f32_smallm(dy, W)),
                ("wgrad dy^T x", lambda: _native.gemm_f32(dy.t(), x), lambda: dy.t() @ x,
                 lambda: _native.gemm_f32_smallm(dy.t(), x))):
            th, tr = t(hip), t(ref)
            ts = t(sm) if m <= 256 else float("nan")
            print(f"m={m:5d} {name:14s} hip {th:7.2f} us ({fl / th / 1e6:6.1f} TF/s)   torch {tr:7.2f} us "
                  f"({fl / tr / 1e6:6.1f} TF/s)   smallm {ts:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
