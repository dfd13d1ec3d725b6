"""Generate tests/golden/outliers.npz from the REFERENCE's own outlier injection (build container only).

    python tests/golden/make_golden_outliers.py

Imports utils/dataset_utils.py in place (tests/golden/refimport.py) and runs
``dataset_utils.inject_outliers(scene, rate)`` (utils/dataset_utils.py:436-461, the call of
train.py:73-81) on CPU scenes under fixed seeds: ``np.random.seed(np_seed)`` for the selection
(np.random.choice in select_outliers) and ``torch.manual_seed(torch_seed)`` for the Gaussian
draws (torch.randn((n_out, 2, 1)), dataset_utils.py:400).  The draws ``z`` are recorded by
re-seeding torch and drawing the same shape (inject_outliers consumes torch's RNG nowhere else).

Cases (synthetic scenes, gasfm_amd.synthetic; pixel M, K^-1 normalisation):
  c1_r10   config-1 scene (m=10, n=200, 3 views per point), rate 0.10
  w_r20    windowed scene m=40, n=3000 (SfM-like locality, ragged view counts), rate 0.20
  w_r35    the same scene, rate 0.35 (several sample / blacklist rounds)
  r_r25    uniform random scene m=24, n=1200, 4 views per point, rate 0.25
  c1_fail  config-1 scene, rate 0.45: every try runs out of free inliers -> None
Saved per case: M, Ns (inputs), seeds and rate, and the result's pixel values at the input edges
(pix_out, from its dense M),
x.indices / x.values of the returned SceneData, the outlier mask over the input edges, z, and
the number of np.random draws (via the RNG state after the call); ``failed`` for None.
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

CASES = (
    ("c1_r10", "config1", 0.10, 101, 102),
    ("w_r20", "windowed", 0.20, 201, 202),
    ("w_r35", "windowed", 0.35, 301, 302),
    ("r_r25", "random", 0.25, 401, 402),
    ("c1_fail", "config1", 0.45, 501, 502),
)


def scene(kind):
    if kind == "config1":
        return synthetic.config1()
    if kind == "windowed":
        return synthetic.windowed_scene(40, 3000, mean_extra=6, seed=9)
    return synthetic.random_scene(24, 1200, 4, seed=3)


def main():
    ref = refimport.load()
    out = {}
    for tag, kind, rate, np_seed, torch_seed in CASES:
        sc = scene(kind)
        M, Ns, Ps = torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns()), torch.from_numpy(sc.Ps_gt())
        data = ref.SceneData.SceneData(M, Ns, Ps, "synthetic_" + kind, calibrated=True)
        idx_in = data.x.indices.numpy()
        np.random.seed(np_seed)
        torch.manual_seed(torch_seed)
        res = ref.dataset_utils.inject_outliers(data, rate)
        # the RNG position after the call: a stand-in for "the same number of draws were made"
        out[f"{tag}_np_next"] = np.random.randint(0, 2**31 - 1, size=4)
        out[f"{tag}_M"], out[f"{tag}_Ns"] = M.numpy(), Ns.numpy()
        out[f"{tag}_params"] = np.array([rate, np_seed, torch_seed], dtype=np.float64)
        if res is None:
            out[f"{tag}_failed"] = np.array(1)
            print(tag, "None (outlier sampling failed)")
            continue
        out[f"{tag}_failed"] = np.array(0)
        M_out = res.M.numpy()
        changed = (M_out[2 * idx_in[0], idx_in[1]] != M.numpy()[2 * idx_in[0], idx_in[1]]) | \
                  (M_out[2 * idx_in[0] + 1, idx_in[1]] != M.numpy()[2 * idx_in[0] + 1, idx_in[1]])
        n_out = int(changed.sum())
        assert n_out == round(rate * idx_in.shape[1])
        torch.manual_seed(torch_seed)
        z = torch.randn((n_out, 2, 1))
        out[f"{tag}_pix_out"] = np.stack([M_out[2 * idx_in[0], idx_in[1]], M_out[2 * idx_in[0] + 1, idx_in[1]]], 1)
        out[f"{tag}_mask"] = changed
        out[f"{tag}_z"] = z.numpy()
        out[f"{tag}_indices"] = res.x.indices.numpy()
        out[f"{tag}_values"] = res.x.values.numpy()
        print(tag, "E", idx_in.shape[1], "outliers", n_out)
    path = os.path.join(HERE, "outliers.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
