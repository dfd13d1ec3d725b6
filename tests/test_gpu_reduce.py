"""gasfm_colsum: one-launch deterministic column sums (last-arriver reduction) vs fp64."""
import pytest
import torch

from gasfm_amd import _native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(0, 7), (1, 1), (3, 5), (127, 64), (128, 64), (7168, 64), (2048, 2176),
                                       (100, 4288), (50_000, 36), (300, 1025)])
def test_colsum_matches_fp64_and_is_deterministic(device, rows, cols):
    g = torch.Generator().manual_seed(rows + 7 * cols)
    A = torch.randn(rows, cols, generator=g, dtype=torch.float64)
    ref = A.sum(0)
    Ad = A.float().to(device)
    outs = [_native.colsum(Ad) for _ in range(3)]  # repeated: the ticket counters must reset
    torch.testing.assert_close(outs[0].double().cpu(), ref, rtol=1e-5, atol=1e-5 * max(1, rows) ** 0.5)
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_colsum_strided_rows(device):
    A = torch.randn(999, 80, device=device)
    torch.testing.assert_close(_native.colsum(A[:, :64]), A[:, :64].sum(0), rtol=1e-5, atol=1e-4)
