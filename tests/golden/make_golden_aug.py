"""Generate tests/golden/scene_aug.npz from the REFERENCE's own per-sample transforms (build container only).

    python tests/golden/make_golden_aug.py

Imports datasets/SceneData.py in place (tests/golden/refimport.py) and runs, on the config-1 scene
(m = 10, each point in 3 of the 10 views), ``sample_data(data, 6)`` after ``np.random.seed(5)``
(6 consecutive views; points left with < 2 views are dropped) and then
``apply_rotational_homography_aug(sampled, 15, 20)`` after ``torch.manual_seed(7)`` (in-plane and
tilt rotations).  pytorch3d is absent offline: ``axis_angle_to_matrix`` is its published formula
as restated in gasfm_amd.scene_device (the product uses the same restatement), so this fixture
pins everything around the rotation matrices: the random draws, the view / point selection, the
homography chain, the zero-reset of invalid points and the graph build.
Saved: the inputs (M, Ns, Ps_gt, seeds, angles) and, for both stages, M, y, x.indices, x.values.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import refimport  # noqa: E402
from gasfm_amd import synthetic  # noqa: E402  (input generation only)
from gasfm_amd.scene_device import _axis_angle_to_matrix  # noqa: E402

NUM_VIEWS, NP_SEED, TORCH_SEED, INPLANE, TILT = 6, 5, 7, 15.0, 20.0


def main():
    ref = refimport.load()
    ref.SceneData.axis_angle_to_matrix = _axis_angle_to_matrix
    sc = synthetic.config1()
    M, Ns, Ps = torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns()), torch.from_numpy(sc.Ps_gt())
    data = ref.SceneData.SceneData(M, Ns, Ps, "synthetic_config1", calibrated=True)
    np.random.seed(NP_SEED)
    s = ref.SceneData.sample_data(data, NUM_VIEWS)
    torch.manual_seed(TORCH_SEED)
    a = ref.SceneData.apply_rotational_homography_aug(s, INPLANE, TILT)
    out = {"M": M, "Ns": Ns, "Ps_gt": Ps,
           "params": np.array([NUM_VIEWS, NP_SEED, TORCH_SEED, INPLANE, TILT], dtype=np.float64)}
    for tag, d in (("s", s), ("a", a)):
        out[f"{tag}_M"], out[f"{tag}_y"] = d.M, d.y
        out[f"{tag}_indices"], out[f"{tag}_values"] = d.x.indices, d.x.values
        print(tag, "M", tuple(d.M.shape), "edges", d.x.indices.shape[1])
    path = os.path.join(HERE, "scene_aug.npz")
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in out.items()})
    print("wrote", path)


if __name__ == "__main__":
    main()
