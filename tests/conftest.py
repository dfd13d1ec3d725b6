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


# multi-process and subprocess tests (spawned ranks, torchrun children) run last: under -x a
# failure there must not keep the single-process kernel / model / config parity suites from running
_RUN_LAST = ("test_distributed.py", "test_dist_train.py")


def pytest_collection_modifyitems(config, items):
    has_gpu = torch.cuda.is_available()
    skip_gpu = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords and not has_gpu:
            it.add_marker(skip_gpu)
    items.sort(key=lambda it: os.path.basename(str(it.fspath)) in _RUN_LAST)  # stable: order kept otherwise


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def device():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def check_grad(got, ref, name, ref32=None, k32=10.0, atol=1e-9):
    """Normwise 1e-3 relative to the fp64 reference (+ atol); where the fp32 oracle itself is worse
    than that (cancellation in tiny gradients), within k32 (10) x the fp32 oracle's own error."""
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    nr = np.linalg.norm(ref)
    bound = 1e-3 * nr + atol
    if ref32 is not None:
        bound = max(bound, k32 * np.linalg.norm(np.asarray(ref32, dtype=np.float64) - ref))
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


def project_grad(key, g):
    """The fixture form of a parameter gradient (tests/golden/make_golden_grads.py): in full up to
    256 elements, else G.reshape(rows, -1) @ probe_vector(key) (rows = first dim, or 16 for a vector)."""
    from oracle.weights import probe_vector
    g = (g.detach().double().cpu() if torch.is_tensor(g) else torch.from_numpy(np.asarray(g, dtype=np.float64)))
    if g.numel() <= 256:
        return g.numpy()
    rows = g.shape[0] if g.dim() >= 2 else (16 if g.numel() % 16 == 0 else 1)
    G = g.reshape(rows, -1)
    return (G @ torch.from_numpy(probe_vector(key, G.shape[1]))).numpy()


def fixture_grad(f, key, tag=""):
    """(reference gradient record, its fp32 counterpart) of parameter ``key`` in fixture f."""
    for suffix in ("", "@r"):
        k = f"grad{tag}/{key}{suffix}"
        if k in f.files:
            k32 = f"grad_fp32/{key}{suffix}"
            return f[k], (f[k32] if k32 in f.files else None)
    raise KeyError(key)


def check_fixture_grads(grads, f, label="", k32=10.0, step_atol=0.0):
    """Every parameter gradient (name -> tensor) against the fixture's fp64 records, at the
    check_grad bound (normwise 1e-3, or k32 x the fp32 reference's own error), plus an absolute
    floor of step_atol x the largest per-tensor gradient norm of the step."""
    recs = {k: fixture_grad(f, k) for k in grads}
    floor = step_atol * max(np.linalg.norm(r) for r, _ in recs.values()) + 1e-9
    for k, g in grads.items():
        ref, ref32 = recs[k]
        check_grad(project_grad(k, g), ref, f"{label}{k}", ref32, k32, atol=floor)
