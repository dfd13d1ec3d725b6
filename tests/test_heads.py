"""View-head decoding (GraphAttnSfMNet.extract_view_outputs) against the reference's own
BaseNet.extract_view_outputs (tests/golden/heads.npz, make_golden_heads.py): calibrated 'quat'
(HIP pose kernel on the GPU), '6d', 'svd' (the reference's geo_utils.project_to_rot), and the
projective head with every normalize_output option.  fp32: |d| <= 1e-5 + 1e-5 |ref|
(the svd variant 1e-4: two independent SVD implementations).
"""
import types

import numpy as np
import pytest
import torch

from conftest import golden
from gasfm_amd.model import GraphAttnSfMNet

CASES = (("quat", True, "quat", None), ("6d", True, "6d", None), ("svd", True, "svd", None),
         ("proj_none", False, "quat", None), ("proj_chir", False, "quat", "Chirality"),
         ("proj_dchir", False, "quat", "Differentiable Chirality"), ("proj_frob", False, "quat", "Frobenius"))


def _decode(tag, calib, rot, norm, device):
    f = golden("heads.npz")
    me = types.SimpleNamespace(calibrated=calib, rot_representation=rot, normalize_output=norm,
                               soft_sign=torch.nn.Softsign())
    x = torch.from_numpy(f[f"{tag}_x"]).to(device).requires_grad_(True)
    Ps = GraphAttnSfMNet.extract_view_outputs(me, x)["Ps_norm"]
    Ps.sum().backward()
    assert torch.isfinite(x.grad).all()
    tol = 1e-4 if tag == "svd" else 1e-5
    np.testing.assert_allclose(Ps.detach().cpu().numpy(), f[f"{tag}_Ps"], rtol=tol, atol=tol)


@pytest.mark.parametrize("tag,calib,rot,norm", CASES)
def test_view_head_decoding_cpu(tag, calib, rot, norm):
    _decode(tag, calib, rot, norm, torch.device("cpu"))


@pytest.mark.gpu
@pytest.mark.parametrize("tag,calib,rot,norm", CASES)
def test_view_head_decoding_gpu(device, tag, calib, rot, norm):
    _decode(tag, calib, rot, norm, device)
