"""gasfm_gemm_bf16 (csrc/gemm_bf16.hip): the bf16 MFMA GEMM of BASELINE config 5's "bf16
projections on MFMA" for the m x 1024 x 1024 camera-side Linear layers
(reference code/models/layers.py:292-320, 352-358, 506-511).

Two references per case:
  - exact: the fp64 product of the bf16-ROUNDED operands.  The kernel multiplies those exactly
    and sums in fp32, so it must agree up to fp32 summation order:
    |C - ref| <= 4 K 2^-24 (|A_bf| |B_bf|)  elementwise (+ the same for Cin / bias adds);
  - the fp32 product of the unrounded operands (what the fp32 path computes): normwise
    |C - ref32| <= 1e-2 |ref32| -- the stated bf16 tolerance of the projection itself
    (operand rounding is 2^-9 relative; random-sign sums keep it near that, measured ~3e-3).
"""
import pytest
import torch

from gasfm_amd import _native

pytestmark = pytest.mark.gpu


def bf16_round(x):
    return x.to(torch.bfloat16).to(torch.float32)


def check(C, a, b, cin=None, bias=None):
    ab, bb = bf16_round(a).double(), bf16_round(b).double()
    ref = ab @ bb
    bound = 4 * a.shape[1] * 2.0 ** -24 * (ab.abs() @ bb.abs())
    if cin is not None:
        ref = ref + cin.double()
        bound = bound + 2.0 ** -23 * (ref.abs() + cin.double().abs())
    if bias is not None:
        ref = ref + bias.double()
        bound = bound + 2.0 ** -23 * (ref.abs() + bias.double().abs())
    err = (C.double() - ref).abs()
    assert bool((err <= bound + 1e-30).all()), f"max excess {(err - bound).max().item():.3e}"
    ref32 = a.double() @ b.double()
    if cin is not None:
        ref32 = ref32 + cin.double()
    if bias is not None:
        ref32 = ref32 + bias.double()
    rel = (C.double() - ref32).norm() / ref32.norm().clamp_min(1e-30)
    assert rel <= 1e-2, f"normwise vs fp32 product {rel:.3e}"
    return rel


@pytest.mark.parametrize("M,N,K", [(1000, 1024, 1024), (37, 64, 100), (1, 2048, 1088), (64, 4, 8), (130, 260, 36)])
def test_forward_form(device, M, N, K):
    """y = x W^T + b (+ skip): A row-major [M,K], B = W.t() (W [N,K] row-major)."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g).to(device)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(device)
    b = torch.randn(N, generator=g).to(device)
    skip = torch.randn(M, N, generator=g).to(device)
    check(_native.gemm_bf16(x, W.t()), x, W.t())
    check(_native.gemm_bf16(x, W.t(), bias=b), x, W.t(), bias=b)
    check(_native.gemm_bf16(x, W.t(), cin=skip, bias=b), x, W.t(), cin=skip, bias=b)


@pytest.mark.parametrize("M,N,K", [(1000, 1024, 1024), (37, 64, 100), (12, 1088, 2048)])
def test_backward_forms(device, M, N, K):
    """dx = dy W (B n-contiguous) and dW = dy^T x (A m-contiguous, K = rows, ragged K)."""
    g = torch.Generator(device="cpu").manual_seed(M + N * 3 + K)
    x = torch.randn(M, K, generator=g).to(device)
    W = torch.randn(N, K, generator=g).to(device)
    dy = torch.randn(M, N, generator=g).to(device)
    check(_native.gemm_bf16(dy, W), dy, W)
    check(_native.gemm_bf16(dy.t(), x), dy.t(), x)


def test_cin_alias_and_empty(device):
    g = torch.Generator(device="cpu").manual_seed(5)
    a = torch.randn(96, 40, generator=g).to(device)
    b = torch.randn(40, 72, generator=g).to(device)
    c = torch.randn(96, 72, generator=g).to(device)
    c0 = c.clone()
    _native.gemm_bf16(a, b, cin=c, out=c)  # in-place accumulate (addmm's C input)
    check(c, a, b, cin=c0)
    z = _native.gemm_bf16(torch.empty(0, 40, device=device), b)
    assert z.shape == (0, 72)
    # K = 0: the product is empty, C = Cin + bias
    e = _native.gemm_bf16(torch.empty(96, 0, device=device), torch.empty(0, 72, device=device), cin=c0)
    torch.testing.assert_close(e, c0, rtol=0, atol=0)


def test_rejects_bad_strides(device):
    a = torch.randn(16, 10, device=device)  # K = 10: float4 runs along k need K % 4 == 0
    b = torch.randn(10, 16, device=device)
    with pytest.raises(RuntimeError, match="float4"):
        _native.gemm_bf16(a, b)
    with pytest.raises(ValueError, match="inner"):
        _native.gemm_bf16(torch.randn(4, 8, device=device), torch.randn(4, 8, device=device))


def test_deterministic(device):
    g = torch.Generator(device="cpu").manual_seed(9)
    a = torch.randn(1000, 1024, generator=g).to(device)
    b = torch.randn(1024, 1024, generator=g).to(device)
    c1 = _native.gemm_bf16(a, b)
    c2 = _native.gemm_bf16(a, b)
    assert torch.equal(c1, c2)
