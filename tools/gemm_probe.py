"""Time the view-side dense GEMM shapes (m x 1024 x 1024, fp32) under torch's BLAS backends.

usage: python tools/gemm_probe.py [m]
Shapes are the three the step issues: Y = X W^T (+b) (forward), dX = dY W, dW = dY^T X; each under
hipBLASLt / rocBLAS fp32 and under the hand-written bf16 MFMA kernel (gasfm_gemm_bf16, fp32 in/out).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gasfm_amd import _native  # noqa: E402


def t(fn, reps=50):
    for _ in range(5):
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
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(m, 1024, device=dev, generator=g)
    W = torch.randn(1024, 1024, device=dev, generator=g)
    b = torch.randn(1024, device=dev, generator=g)
    dY = torch.randn(m, 1024, device=dev, generator=g)
    flop = 2 * m * 1024 * 1024
    for lib in ("cublaslt", "cublas"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:  # noqa: BLE001
            print(lib, "unavailable:", e)
            continue
        res = {
            "fwd addmm X W^T + b": t(lambda: torch.addmm(b, X, W.t())),
            "bwd dX = dY W": t(lambda: torch.mm(dY, W)),
            "bwd dW = dY^T X": t(lambda: torch.mm(dY.t(), X)),
        }
        for k, us in res.items():
            print(f"{lib:9s} m={m} {k:22s} {us:7.2f} us  {flop / us / 1e6:6.1f} TF/s", flush=True)
    torch.backends.cuda.preferred_blas_library("cublaslt")
    skip = torch.randn(m, 1024, device=dev, generator=g)
    res = {
        "fwd X W^T + b + skip": t(lambda: _native.gemm_bf16(X, W.t(), cin=skip, bias=b)),
        "bwd dX = dY W": t(lambda: _native.gemm_bf16(dY, W)),
        "bwd dW = dY^T X": t(lambda: _native.gemm_bf16(dY.t(), X)),
    }
    for k, us in res.items():
        print(f"{'gemm_bf16':9s} m={m} {k:22s} {us:7.2f} us  {flop / us / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
