"""Generate tests/golden/heads.npz from the REFERENCE's own view-head decoding (build container only).

    python tests/golden/make_golden_heads.py

Calls BaseNet.extract_view_outputs (code/models/baseNet.py:38-85) unbound, on a stand-in ``self``
carrying the attributes it reads (calibrated, rot_representation, normalize_output, soft_sign),
for every head variant: calibrated 'quat' / '6d' / 'svd' and projective with normalize_output
None / 'Chirality' / 'Differentiable Chirality' / 'Frobenius'.  'svd' runs the reference's
geo_utils.project_to_rot; pytorch3d (absent offline) is restated from its published formulas for
'quat' and '6d' (the product uses the same restatements: gasfm_amd.model), so for those two the
rotation function itself is "parity unpinned" and everything around it is pinned.
Inputs: seeded random head outputs x [m, out_dim], m = 16.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refimport  # noqa: E402
from gasfm_amd.model import rotation_6d_to_matrix  # noqa: E402

CASES = (("quat", True, "quat", None, 7), ("6d", True, "6d", None, 9), ("svd", True, "svd", None, 12),
         ("proj_none", False, "quat", None, 12), ("proj_chir", False, "quat", "Chirality", 12),
         ("proj_dchir", False, "quat", "Differentiable Chirality", 12), ("proj_frob", False, "quat", "Frobenius", 12))


def main():
    ns = refimport.load()
    import importlib
    base = importlib.import_module("models.baseNet")
    base.py3d_trans.rotation_6d_to_matrix = rotation_6d_to_matrix
    g = torch.Generator().manual_seed(3)
    out = {}
    for tag, calib, rot, norm, d in CASES:
        x = torch.randn((16, d), generator=g, dtype=torch.float32)
        fake = types.SimpleNamespace(calibrated=calib, rot_representation=rot, normalize_output=norm,
                                     soft_sign=torch.nn.Softsign())
        Ps = base.BaseNet.extract_view_outputs(fake, x)["Ps_norm"]
        out[f"{tag}_x"], out[f"{tag}_Ps"] = x.numpy(), Ps.numpy()
        print(tag, tuple(Ps.shape))
    del ns
    path = os.path.join(HERE, "heads.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
