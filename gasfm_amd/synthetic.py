"""Synthetic camera/point scenes for the BASELINE configs (no datasets ship offline).

config 1 (BASELINE.json configs[0]): m=10, n=200, every point in
    3 distinct random cameras, numpy default_rng(0), pixels U(1,1000),
    K = [[800,0,500],[0,800,500],[0,0,1]], Ps_gt = [I|0].
config 4 (configs[3]): m=1000, n=200,000, point j visible in
    k_j = clip(2 + Poisson(18), 2, m) distinct cameras drawn from a contiguous
    window of 2*k_j cameras around a random centre (SfM-like locality),
    default_rng(4); every camera keeps >= 8 points (constants.py:6).  E ~ 4.0M.

A scene is returned in sparse form (cam, pt, pixel xy) so that config 4 never
materialises the dense 2m x n measurement matrix; ``dense_M`` builds it for
small scenes (the reference's SceneData input, Euclidean.py:22-39).
"""
from dataclasses import dataclass

import numpy as np

K_DEFAULT = np.array([[800.0, 0.0, 500.0], [0.0, 800.0, 500.0], [0.0, 0.0, 1.0]])


@dataclass
class SyntheticScene:
    m: int
    n: int
    cam: np.ndarray   # [E] int64, cam-major sorted (then point)
    pt: np.ndarray    # [E] int64
    xy: np.ndarray    # [E, 2] float32 pixel coordinates
    K: np.ndarray     # [3, 3]

    @property
    def num_edges(self):
        return int(self.cam.shape[0])

    def normalized_values(self):
        """(N @ [x, y, 1])[:2] with N = K^-1 (Euclidean.py:30-32, geo_utils.normalize_M)."""
        N = np.linalg.inv(self.K)
        h = np.concatenate([self.xy.astype(np.float64), np.ones((self.num_edges, 1))], axis=1)
        v = h @ N.T
        return v[:, :2].astype(np.float32)

    def dense_M(self):
        M = np.zeros((2 * self.m, self.n), dtype=np.float32)
        M[2 * self.cam, self.pt] = self.xy[:, 0]
        M[2 * self.cam + 1, self.pt] = self.xy[:, 1]
        return M

    def Ns(self):
        return np.repeat(np.linalg.inv(self.K)[None].astype(np.float32), self.m, axis=0)

    def Ps_gt(self):
        P = np.zeros((self.m, 3, 4), dtype=np.float32)
        P[:, :3, :3] = np.eye(3, dtype=np.float32)
        return P


def _sorted(m, n, cam, pt, rng):
    order = np.lexsort((pt, cam))
    cam, pt = cam[order].astype(np.int64), pt[order].astype(np.int64)
    xy = rng.uniform(1.0, 1000.0, size=(cam.shape[0], 2)).astype(np.float32)
    return SyntheticScene(m, n, cam, pt, xy, K_DEFAULT.copy())


def random_scene(m, n, views_per_point, seed, window=None):
    """Each point in `views_per_point` distinct cameras (uniform, or inside a window)."""
    rng = np.random.default_rng(seed)
    cams = np.empty((n, views_per_point), dtype=np.int64)
    for j in range(n):
        cams[j] = rng.choice(m, size=views_per_point, replace=False)
    pt = np.repeat(np.arange(n, dtype=np.int64), views_per_point)
    return _sorted(m, n, cams.reshape(-1), pt, rng)


def config1():
    return random_scene(10, 200, 3, seed=0)


def windowed_scene(m, n, mean_extra=18, seed=4, min_pts_per_cam=8):
    """config-4 generator (vectorised over points grouped by their view count)."""
    rng = np.random.default_rng(seed)
    k = np.clip(2 + rng.poisson(mean_extra, size=n), 2, m).astype(np.int64)
    centre = rng.integers(0, m, size=n)
    cam_parts, pt_parts = [], []
    for kv in np.unique(k):
        idx = np.nonzero(k == kv)[0]
        w = min(2 * int(kv), m)
        # kv distinct offsets out of a window of w cameras: argsort of random keys
        keys = rng.random((idx.shape[0], w))
        offs = np.argsort(keys, axis=1)[:, :kv] - w // 2
        cams = (centre[idx, None] + offs) % m
        cam_parts.append(cams.reshape(-1))
        pt_parts.append(np.repeat(idx, kv))
    cam = np.concatenate(cam_parts)
    pt = np.concatenate(pt_parts)
    counts = np.bincount(cam, minlength=m)
    if counts.min() < min_pts_per_cam:
        # top up starving cameras with extra observations of random points not yet seen
        extra_c, extra_p = [], []
        seen = set(zip(cam.tolist(), pt.tolist())) if cam.shape[0] < 5_000_000 else None
        for c in np.nonzero(counts < min_pts_per_cam)[0]:
            need = min_pts_per_cam - counts[c]
            while need > 0:
                p = int(rng.integers(0, n))
                if seen is not None and (int(c), p) in seen:
                    continue
                extra_c.append(c)
                extra_p.append(p)
                if seen is not None:
                    seen.add((int(c), p))
                need -= 1
        cam = np.concatenate([cam, np.asarray(extra_c, dtype=np.int64)])
        pt = np.concatenate([pt, np.asarray(extra_p, dtype=np.int64)])
    return _sorted(m, n, cam, pt, rng)


def config4(m=1000, n=200_000, seed=4):
    return windowed_scene(m, n, seed=seed)


CONFIG2_M, CONFIG2_N, CONFIG2_EXTRA = 133, 23674, 4


def config2_standin(seed=2):
    """Synthetic stand-in for BASELINE config 2's single scene, AlcatrazCourtyard
    (optim_euc_gasfm.conf:6; single_scene_optimization.py:15-123).  The dataset file
    (datasets/Euclidean/AlcatrazCourtyard.npz, README.md:70-76) is not available offline, so its
    size is taken from the published dataset statistics as recalled (133 views, 23,674 points:
    UNVERIFIED here) and the track length, unknown offline, is set to 2 + Poisson(4) views per
    point (~6): E ~ 142k.  Values and visibility are synthetic (windowed SfM-like generator)."""
    return windowed_scene(CONFIG2_M, CONFIG2_N, mean_extra=CONFIG2_EXTRA, seed=seed)


def scaled_config4(scale, seed=4):
    """config 4 with m and n scaled by `scale` (parity tests at oracle-friendly sizes)."""
    return windowed_scene(max(16, int(1000 * scale)), max(64, int(200_000 * scale)), seed=seed)


def rotation_look_at(center, target=np.zeros(3), up=np.array([0.0, 0.0, 1.0])):
    """Camera-to-world orientation R (columns: camera x, y, z axes in world coordinates) of a camera
    at ``center`` looking at ``target``; P = K R^T [I | -center] (geo_utils.get_camera_matrix)."""
    z = target - center
    z = z / np.linalg.norm(z)
    x = np.cross(z, up)
    x = x / np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=1)


def ba_scene(m, n, views_per_point, noise_px=0.0, seed=0, radius=4.0, f=800.0):
    """Bundle-adjustment test scene (BASELINE config-4 style windowed visibility): m cameras on a
    circle of ``radius`` looking at points uniform in [-1, 1]^3, point j seen by
    ``views_per_point`` consecutive cameras; returns dict(xs [m, n, 2] pixels (0 = unseen),
    Rs, ts (camera centres), Ks, Xs [n, 3]) -- the euc_ba inputs (ba_functions.py:6)."""
    rng = np.random.default_rng(seed)
    ang = np.linspace(0, 2 * np.pi, m, endpoint=False)
    ts = np.stack([radius * np.cos(ang), radius * np.sin(ang), 0.3 * rng.standard_normal(m)], 1)
    Rs = np.stack([rotation_look_at(c) for c in ts])
    Ks = np.repeat(np.array([[f, 0.0, 500.0], [0.0, f, 500.0], [0.0, 0.0, 1.0]])[None], m, axis=0)
    Xs = rng.uniform(-1, 1, size=(n, 3))
    xs = np.zeros((m, n, 2))
    start = rng.integers(0, m, size=n)
    j = np.repeat(np.arange(n), views_per_point)
    c = (np.repeat(start, views_per_point) + np.tile(np.arange(views_per_point), n)) % m
    q = np.einsum("eij,ej->ei", Ks[c] @ Rs[c].transpose(0, 2, 1), Xs[j] - ts[c])
    xs[c, j] = q[:, :2] / q[:, 2:3]
    if noise_px:
        xs[c, j] += noise_px * rng.standard_normal((c.shape[0], 2))
    return {"xs": xs, "Rs": Rs, "ts": ts, "Ks": Ks, "Xs": Xs}
