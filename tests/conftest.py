import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP path")
    config.addinivalue_line("markers", "reference: needs /root/reference (build container only)")


def pytest_collection_modifyitems(config, items):
    has_gpu = torch.cuda.is_available()
    skip_gpu = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords and not has_gpu:
            it.add_marker(skip_gpu)


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def device():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def check_grad(got, ref, name, ref32=None):
    """Normwise 1e-3 relative to the fp64 reference; where the fp32 oracle itself is worse than
    that (cancellation in tiny gradients), within 10x of the fp32 oracle's own error."""
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    nr = np.linalg.norm(ref)
    bound = 1e-3 * nr + 1e-9
    if ref32 is not None:
        bound = max(bound, 10 * np.linalg.norm(np.asarray(ref32, dtype=np.float64) - ref))
    err = np.linalg.norm(got - ref)
    assert err <= bound, f"{name}: normwise {err:.3e} vs |ref| {nr:.3e} (bound {bound:.3e})"


def oracle_grads(sd64, sc, cP, cX):
    """fp64 and fp32 oracle parameter gradients of sum(Ps*cP) + sum(pts3D*cX) on a synthetic scene."""
    from oracle import gasfm_ref, scenes
    g = scenes.graph_from_edges(sc.cam, sc.pt, sc.m, sc.n)
    vals = torch.from_numpy(sc.normalized_values())
    out = {}
    for dt in (torch.float64, torch.float32):
        sd = {k: v.to(dt).clone().requires_grad_(True) for k, v in sd64.items()}
        r = gasfm_ref.forward(sd, vals.to(dt), g, dtype=dt)
        ((r["Ps_norm"] * cP.to(dt)).sum() + (r["pts3D"] * cX.to(dt)).sum()).backward()
        out[dt] = ({k: (v.grad if v.grad is not None else torch.zeros_like(v)).double().numpy()
                    for k, v in sd.items()}, r)
    return out[torch.float64], out[torch.float32]
