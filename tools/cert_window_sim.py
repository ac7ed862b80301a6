"""CPU model of k_icp_nn's steady state on a bench pair: which source points
lose their two-nearest certificate in each iteration, how wide the pixel
window their search stages is, and how those lanes fall into wavefronts
(64 consecutive points of the Morton-sorted source, as the kernel reads
them).  The poses are the oracle's REF loop (align_icp.cpp:92-153); the
neighbour search is scipy's exact kd-tree (ties aside, the same answers).

    python tools/cert_window_sim.py [--pair 1] [--iters 128]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np
from scipy.spatial import cKDTree

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402


def morton_order(p):
    lo, hi = p.min(0), p.max(0)
    q = ((p - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.uint64)

    def spread(x):
        x = x & 0x3FF
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        x = (x | (x << 2)) & 0x09249249
        return x
    code = spread(q[:, 0]) | (spread(q[:, 1]) << np.uint64(1)) | (spread(q[:, 2]) << np.uint64(2))
    return np.argsort(code, kind="stable")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pair", type=int, default=1)
    ap.add_argument("--iters", type=int, default=128)
    ap.add_argument("--cap", type=float, default=20.0)
    a = ap.parse_args()
    K = driver.intrinsics(640, 480)
    sc = driver.SyntheticScene(0)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    dst = O.unproject(sc.render(sc.trajectory(a.pair - 1), K, noise_seed=a.pair - 1), K4)
    src = O.unproject(sc.render(sc.trajectory(a.pair), K, noise_seed=a.pair), K4)
    O.set_threads(8)
    _, _, _, tr = O.align_icp(src, dst, a.iters, tree=O.KDTree(dst), trace=True, sum_mode=0)
    poses = [np.eye(4, dtype=np.float32)] + list(tr["pose"][:-1])  # the pose iteration k transforms with
    order = morton_order(src)
    s = src[order].astype(np.float64)
    tree = cKDTree(dst)
    n = len(s)
    p_idx = np.full(n, -1)
    q0 = np.zeros((n, 3))
    g = np.zeros(n)
    fx = abs(K.fx)
    print(f"pair {a.pair}: n={n} m={len(dst)}")
    for k in range(a.iters):
        T = poses[k].astype(np.float64)
        q = s @ T[:3, :3].T + T[:3, 3]
        have = p_idx >= 0
        dp = np.linalg.norm(q - dst[np.maximum(p_idx, 0)], axis=1)
        moved = np.linalg.norm(q - q0, axis=1)
        cert = have & (dp + moved < g)
        need = ~cert
        d, j = tree.query(q[need], k=2)
        # the window of the seed distance r = |q - p_old| (cold: the search's own)
        r = np.where(have[need], dp[need], d[:, 0])
        z = np.maximum(q[need, 2], 1e-3)
        half = fx * r / np.maximum(z - r, 1e-3)
        p_idx[need] = j[:, 0]
        q0[need] = q[need]
        g[need] = d[:, 1] - 1e-5 * d[:, 1]
        if k in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 127):
            w = need.reshape(-1)[: n // 64 * 64].reshape(-1, 64)
            per_wave = w.sum(1)
            hw = np.zeros(n)
            hw[need] = half
            wmax = hw[: n // 64 * 64].reshape(-1, 64).max(1)
            qs = np.percentile(half, [50, 90, 99]) if need.any() else [0, 0, 0]
            print(f"it {k:3d}: searched {need.sum():6d} ({100 * need.mean():.2f}%), waves with a search "
                  f"{100 * (per_wave > 0).mean():5.1f}% (mean {per_wave[per_wave > 0].mean() if (per_wave > 0).any() else 0:.1f} "
                  f"lanes), half-width p50/p90/p99 {qs[0]:.1f}/{qs[1]:.1f}/{qs[2]:.1f} px, "
                  f"> cap {int((half > a.cap).sum())}; wave max-half p50/p90 "
                  f"{np.percentile(wmax[per_wave > 0], 50) if (per_wave > 0).any() else 0:.1f}/"
                  f"{np.percentile(wmax[per_wave > 0], 90) if (per_wave > 0).any() else 0:.1f}; "
                  f"waves whose max half <= 1 / 2 px: {100 * ((wmax <= 1) & (per_wave > 0)).mean():.1f}% / "
                  f"{100 * ((wmax <= 2) & (per_wave > 0)).mean():.1f}%", flush=True)


if __name__ == "__main__":
    main()
