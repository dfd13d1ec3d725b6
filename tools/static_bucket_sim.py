"""The bucket policy of gasfm_amd/static_batch.py on config-3-shaped batches, on the CPU.

usage: python tools/static_bucket_sim.py [batches]

12 synthetic training scenes (m = 100, n = 20k windowed), batches of 4 sampled to 10-20 views on
the host (no augmentation: the graph sizes are what the buckets see), each batch placed as
StaticTrainer._bucket places it.  Prints the bucket per batch, the number of buckets and the mean
padding (bucket edges / batch edges).
"""
import sys, time
import numpy as np, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import gasfm_amd
from gasfm_amd import synthetic, static_batch
from gasfm_amd.scene import SceneData
from gasfm_amd.scene_device import sample_indices
np.random.seed(0)
scenes = []
for i in range(12):
    sc = synthetic.windowed_scene(100, 20000, seed=100 + i)
    scenes.append((torch.from_numpy(sc.dense_M()), torch.from_numpy(sc.Ns()), torch.from_numpy(sc.Ps_gt())))
def prep(s):
    M, Ns, y = s
    idx = sample_indices(len(y), int(np.random.randint(10, 21)), adjacent=True)
    m_idx = np.sort(np.concatenate((2 * idx, 2 * idx + 1)))
    Mi = M.numpy()[m_idx]
    xs = Mi.reshape(len(idx), 2, -1)
    keep = ((np.abs(xs).sum(1) != 0).sum(0) >= 2)
    return SceneData(torch.from_numpy(np.ascontiguousarray(Mi[:, keep])), Ns[idx], y[idx], "s")
buckets = []
wastes = []
t0 = time.time()
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 60):
    datas = [prep(scenes[int(i)]) for i in np.random.choice(12, int(__import__("os").environ.get("SIM_BATCH", "4")), replace=False)]
    st = static_batch.BatchStats(datas)
    why = st.expressible()
    if why:
        print("not expressible", why); continue
    best = None
    for c in buckets:
        if c.pad(st) is not None and c.waste_ok(st) and (best is None or c.E < best.E):
            best = c
    new = best is None
    if new:
        best = static_batch.Caps.for_batch(st); buckets.append(best)
    wastes.append(best.E / st.E)
    print(it, "E", st.E, "N", st.N, "M", st.M, "pieces", st.pieces, "kp min", min(st.kp), "-> bucket", best.key(), "new" if new else "", f"waste {best.E/st.E:.3f}", flush=True)
print("buckets", len(buckets), "mean waste", np.mean(wastes), time.time() - t0)
