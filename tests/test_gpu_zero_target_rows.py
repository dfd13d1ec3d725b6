"""gatv2.zero_target_rows (the stateless targets' lin_r(0) == bias broadcast, dataset_utils.py:569-571)
returns rows that do not alias the bias parameter: an in-place update of the bias after
the forward leaves the saved XR unchanged and its backward still works; the bias gradient is the
column sum of the rows' gradient (exactly, in fp32), the weight's gradient zero."""
import pytest
import torch

from gasfm_amd import gatv2

pytestmark = pytest.mark.gpu


def test_zero_target_rows_do_not_alias_bias(device):
    torch.manual_seed(0)
    lin = torch.nn.Linear(32, 32).to(device)
    n = 1000
    xr = gatv2.zero_target_rows(lin, n, lin.weight)
    assert xr.shape == (n, 32)
    assert xr.untyped_storage().data_ptr() != lin.bias.untyped_storage().data_ptr()
    before = xr.detach().clone()
    torch.testing.assert_close(before, lin.bias.detach().expand(n, -1), rtol=0, atol=0)
    with torch.no_grad():
        lin.bias.add_(1.0)  # an optimizer step between forward and backward
    torch.testing.assert_close(xr.detach(), before, rtol=0, atol=0)
    g = torch.randn(n, 32, device=device)
    (xr * g).sum().backward()
    torch.cuda.synchronize()
    torch.testing.assert_close(lin.bias.grad, g.double().sum(0).float(), rtol=1e-5, atol=1e-5)
    assert torch.count_nonzero(lin.weight.grad) == 0
