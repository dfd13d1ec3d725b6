"""gasfm_gemm_f32 (csrc/gemm_f32.hip): the fp32 MFMA GEMM of the camera-side m x 1024 x 1024
Linear layers (reference code/models/layers.py:292-320, 352-358, 506-511), at m = 1000 (one GPU)
and m = 125 (a camera shard of 8 GPUs), in all three Linear forms (y = x W^T, dx = dy W,
dW = dy^T x) with the fused bias / Cin epilogue.

Reference: the fp64 product.  v_mfma_f32_16x16x4_f32 forms exact products and the kernel sums in
fp32, so the error is fp32 summation error: |C - ref| <= 4 K 2^-24 (|A| |B|) elementwise (+ one
rounding per Cin / bias add) -- the bound a k-ordered fp32 fma chain meets.
"""
import pytest
import torch

from gasfm_amd import _native

pytestmark = pytest.mark.gpu


def check(C, a, b, cin=None, bias=None):
    ad, bd = a.double(), b.double()
    ref = ad @ bd
    bound = 4 * a.shape[1] * 2.0 ** -24 * (ad.abs() @ bd.abs())
    if cin is not None:
        ref = ref + cin.double()
        bound = bound + 2.0 ** -23 * (ref.abs() + cin.double().abs())
    if bias is not None:
        ref = ref + bias.double()
        bound = bound + 2.0 ** -23 * (ref.abs() + bias.double().abs())
    err = (C.double() - ref).abs()
    assert bool((err <= bound + 1e-30).all()), f"max excess {(err - bound).max().item():.3e}"


SHAPES = [(1000, 1024, 1024), (125, 1024, 1024), (128, 1024, 1088), (37, 64, 100), (1, 2048, 1088),
          (64, 4, 8), (130, 260, 36), (7, 32, 1024)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_forward_form(device, M, N, K):
    """y = x W^T + b (+ skip): A row-major [M,K], B = W.t() (W [N,K] row-major)."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g).to(device)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(device)
    b = torch.randn(N, generator=g).to(device)
    skip = torch.randn(M, N, generator=g).to(device)
    check(_native.gemm_f32(x, W.t()), x, W.t())
    check(_native.gemm_f32(x, W.t(), bias=b), x, W.t(), bias=b)
    check(_native.gemm_f32(x, W.t(), cin=skip, bias=b), x, W.t(), cin=skip, bias=b)
    acc = skip.clone()  # in place: out is cin
    _native.gemm_f32(x, W.t(), cin=acc, out=acc)
    check(acc, x, W.t(), cin=skip)


@pytest.mark.parametrize("M,N,K", [(1000, 1024, 1024), (125, 1024, 1024), (37, 64, 100), (12, 1088, 2048)])
def test_input_grad_form(device, M, N, K):
    """dx = dy W: A = dy [M,K] row-major, B = W [K,N] row-major (n-contiguous)."""
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N)
    dy = torch.randn(M, K, generator=g).to(device)
    W = torch.randn(K, N, generator=g).to(device)
    skip = torch.randn(M, N, generator=g).to(device)
    check(_native.gemm_f32(dy, W), dy, W)
    check(_native.gemm_f32(dy, W, cin=skip), dy, W, cin=skip)


@pytest.mark.parametrize("R,O,I", [(1000, 1024, 1024), (125, 1024, 1024), (100, 64, 36), (2048, 12, 1088), (125, 32, 1024)])
def test_weight_grad_form(device, R, O, I):
    """dW = dy^T x: A = dy.t() (m-contiguous), B = x [R, I] row-major (n-contiguous), K = R."""
    g = torch.Generator(device="cpu").manual_seed(R + O + I)
    dy = torch.randn(R, O, generator=g).to(device)
    x = torch.randn(R, I, generator=g).to(device)
    check(_native.gemm_f32(dy.t(), x), dy.t(), x)


def test_deterministic_and_torch_close(device):
    g = torch.Generator(device="cpu").manual_seed(5)
    a = torch.randn(125, 1024, generator=g).to(device)
    b = torch.randn(1024, 1024, generator=g).to(device)
    c1 = _native.gemm_f32(a, b)
    c2 = _native.gemm_f32(a, b)
    assert torch.equal(c1, c2)
    torch.testing.assert_close(c1, a @ b, rtol=1e-4, atol=1e-3)


def test_rejects_bad_operands(device):
    a = torch.randn(8, 6, device=device)  # K = 6: no float4 runs along k
    with pytest.raises(Exception):
        _native.gemm_f32(a, torch.randn(6, 8, device=device).t().contiguous().t())
    with pytest.raises(ValueError):
        _native.gemm_f32(torch.randn(8, 8, device=device), torch.randn(4, 8, device=device))
