"""Calibrated camera head (csrc/pose_head.hip) vs the fp64 reference formula.

Reference: baseNet.extract_view_outputs, rot_representation 'quat' (code/models/baseNet.py:38-56):
pytorch3d quaternion_to_matrix (restated as gasfm_amd.model.quaternion_to_matrix) and
torch.cat with the translation.  Tolerance: 1e-6 absolute on outputs and gradients (unit-scale
quaternions, fp32 arithmetic).
"""
import pytest
import torch

from gasfm_amd.model import QuatPoseFn, quaternion_to_matrix

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m", [1, 7, 1000])
def test_pose_head_matches_fp64(device, m):
    g = torch.Generator().manual_seed(m)
    x64 = torch.randn(m, 7, generator=g, dtype=torch.float64)
    dP = torch.randn(m, 3, 4, generator=g, dtype=torch.float64)
    xr = x64.clone().requires_grad_(True)
    ref = torch.cat((quaternion_to_matrix(xr[:, :4]), xr[:, -3:].unsqueeze(-1)), dim=-1)
    ref.backward(dP)
    x = x64.float().to(device).requires_grad_(True)
    out = QuatPoseFn.apply(x)
    out.backward(dP.float().to(device))
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(x.grad.double().cpu(), xr.grad, rtol=1e-4, atol=1e-5)
