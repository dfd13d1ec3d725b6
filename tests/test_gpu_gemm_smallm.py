"""The small-row-count fp32 GEMMs (csrc/gemm_smallm.hip, gasfm_gemm_f32_smallm) against an fp64 torch
reference: the three products of the camera-side Linear layers on a camera-sharded rank (125 rows
at config 4 on 8 GPUs) and a training batch (~60 rows), with the fused bias / skip epilogue and the
in-place skip.  Tolerance (fp32 MFMA, k-ordered fp32 sums over K <= 1024 vs fp64):
|d| <= 1e-4 |ref|_max + 1e-6, the products' inputs being O(1).  The view-chain dispatch
(view_block._mm) is checked to take this kernel at m <= GASFM_SMALLM_ROWS.
"""
import pytest
import torch

from gasfm_amd import _native, view_block

pytestmark = pytest.mark.gpu


def _close(got, ref):
    ref = ref.double()
    err = float((got.double() - ref).abs().max())
    assert err <= 1e-4 * float(ref.abs().max()) + 1e-6, err


@pytest.mark.parametrize("M", [1, 17, 60, 125, 256])
@pytest.mark.parametrize("K", [128, 1024])
def test_xwt_and_xw(device, M, K):
    g = torch.Generator(device=device).manual_seed(M * 7 + K)
    N = 1024
    x = torch.randn(M, K, generator=g, device=device)
    W = torch.randn(N, K, generator=g, device=device) / K ** 0.5
    b = torch.randn(N, generator=g, device=device)
    skip = torch.randn(M, N, generator=g, device=device)
    y = _native.gemm_f32_smallm(x, W.t())
    assert y is not None
    _close(y, x.double() @ W.double().t())
    y = _native.gemm_f32_smallm(x, W.t(), bias=b)
    _close(y, x.double() @ W.double().t() + b.double())
    ref = skip.double() + x.double() @ W.double().t()
    y = _native.gemm_f32_smallm(x, W.t(), cin=skip, out=skip)  # in place, as ViewTailFn's MLP
    assert y is skip
    _close(y, ref)
    # dx = dy W with W [K_out = K, N]
    W2 = torch.randn(K, N, generator=g, device=device) / K ** 0.5
    y = _native.gemm_f32_smallm(x, W2)
    _close(y, x.double() @ W2.double())


@pytest.mark.parametrize("K", [1, 16, 60, 125, 256])
def test_wgrad(device, K):
    g = torch.Generator(device=device).manual_seed(K)
    dy = torch.randn(K, 1024, generator=g, device=device)
    x = torch.randn(K, 512, generator=g, device=device)
    y = _native.gemm_f32_smallm(dy.t(), x)
    assert y is not None and y.shape == (1024, 512)
    _close(y, dy.double().t() @ x.double())


def test_unsupported_forms_fall_back(device):
    a = torch.randn(8, 100, device=device)  # K not a multiple of the K-slicing
    assert _native.gemm_f32_smallm(a, torch.randn(64, 100, device=device).t()) is None
    a = torch.randn(8, 64, device=device)
    assert _native.gemm_f32_smallm(a, torch.randn(64, 48, device=device)) is None  # N % 32 != 0
    assert _native.gemm_f32_smallm(a, torch.randn(64, 64, device=device), bias=torch.zeros(64, device=device)) is None


def test_view_chain_dispatch(device):
    """view_block._mm takes the small-M kernels for the three products at m = 125 (dispatch seen
    through the results' bitwise equality with direct calls)."""
    g = torch.Generator(device=device).manual_seed(3)
    m, D = 125, 1024
    h = torch.randn(m, D, generator=g, device=device)
    Wm = torch.randn(D, D, generator=g, device=device) / 32
    dv = torch.randn(m, D, generator=g, device=device)
    assert m <= view_block.SMALLM_ROWS
    assert torch.equal(view_block._mm(h, Wm.t()), _native.gemm_f32_smallm(h, Wm.t()))
    assert torch.equal(view_block._mm(dv, Wm), _native.gemm_f32_smallm(dv, Wm))
    assert torch.equal(view_block._mm(dv.t(), h), _native.gemm_f32_smallm(dv.t(), h))
