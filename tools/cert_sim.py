"""CPU simulation of the ICP loop's certificates on the bench pair (640x480
frames 0 -> 1): per iteration, the fraction of source points whose
certificate fails (the search queue) with K = 1, 2, 4 kept candidates --
a candidate list certified while min_j |q - p_j| + |q - q0| < r_{K+1}(q0).
Poses from the oracle's trace; neighbours from scipy's cKDTree.
  python tools/cert_sim.py"""
import sys
from pathlib import Path

import numpy as np
from scipy.spatial import cKDTree

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
da = sc.render(sc.trajectory(0), K, noise_seed=1)
db = sc.render(sc.trajectory(1), K, noise_seed=2)
K4 = [K.fx, K.fy, K.cx, K.cy]
dst = O.unproject(da, K4).astype(np.float64)
src = O.unproject(db, K4).astype(np.float64)
O.set_threads(8)
_, _, _, tr = O.align_icp(src, dst, 128, trace=True, sum_mode=1)
poses = [np.eye(4)] + [p.astype(np.float64) for p in tr["pose"][:-1]]
tree = cKDTree(dst)
KS = (1, 2, 4)
state = {k: None for k in KS}
rows = []
for it, P in enumerate(poses):
    Q = src @ P[:3, :3].T + P[:3, 3]
    d, idx = tree.query(Q, k=5, workers=8)
    row = [it]
    for k in KS:
        st = state[k]
        if st is None:
            fail = np.ones(len(Q), bool)
            st = {"q0": Q.copy(), "c": idx[:, :k].copy(), "g": d[:, k].copy()}
        else:
            delta = np.linalg.norm(Q - st["q0"], axis=1)
            dm = np.min(np.linalg.norm(Q[:, None, :] - dst[st["c"]], axis=2), axis=1)
            fail = ~(dm + delta < st["g"])
            st["q0"][fail] = Q[fail]
            st["c"][fail] = idx[fail, :k]
            st["g"][fail] = d[fail, k]
        state[k] = st
        row.append(fail.mean())
    rows.append(row)
    if it in (0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 127):
        print(f"{it:4d} " + " ".join(f"K{k}:{v:7.4f}" for k, v in zip(KS, row[1:])), flush=True)
a = np.array(rows)
print("mean queue fraction over iterations 1..127:", {k: round(float(a[1:, j + 1].mean()), 4)
                                                      for j, k in enumerate(KS)})
