"""How many correspondences change from one ICP iteration to the next.

The reference's d-bar chains (align_icp.cpp:113, `dst_mean += dst.GetPoint(j)`)
depend only on the neighbour indices; an iteration whose indices equal the
previous one's has the same d-bar bit for bit.  This tool runs the oracle's
AlignIcp3d restatement on a 640x480 pair of the bench stream with a trace,
recomputes every iteration's neighbours from the traced poses and prints,
per iteration, the number of changed indices and how they spread over the
sequential sums' 16-element windows, 4096-element tiles and 256-element
groups (CPU only; the oracle's arithmetic is the kernels' bit for bit).

    python tools/nbr_changes.py [--width 640 --height 480 --iters 128 --pair 0]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle import oracle as O  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--iters", type=int, default=128)
    ap.add_argument("--pair", type=int, default=0)
    a = ap.parse_args()
    K = driver.intrinsics(a.width, a.height)
    sc = driver.SyntheticScene(0)
    k = a.pair
    da = sc.render(sc.trajectory(k), K, noise_seed=k)
    db = sc.render(sc.trajectory(k + 1), K, noise_seed=k + 1)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    dst = O.unproject(da, K4)
    src = O.unproject(db, K4)
    tree = O.KDTree(dst, 16)
    _, _, _, tr = O.align_icp(src, dst, a.iters, tree=tree, trace=True)
    n = len(src)
    prev = None
    print(f"n {n} m {len(dst)}")
    print(" it  changed  windows16  groups256  tiles4096 first_pos")
    tot = 0
    zero = 0
    for it in range(a.iters):
        T = np.eye(4, dtype=np.float32) if it == 0 else tr["pose"][it - 1]
        q = O.transform_points(T, src)
        idx, _ = tree.query(q)
        if prev is not None:
            ch = np.nonzero(idx != prev)[0]
            tot += len(ch)
            zero += int(len(ch) == 0)
            w = len(np.unique(ch // 16))
            g = len(np.unique(ch // 256))
            t = len(np.unique(ch // 4096))
            print(f"{it:3d} {len(ch):8d} {w:10d} {g:10d} {t:10d} {ch[0] if len(ch) else -1:9d}")
        prev = idx
    print(f"iterations with no change: {zero} of {a.iters - 1}; changed indices total {tot}")


if __name__ == "__main__":
    main()
