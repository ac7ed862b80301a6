"""Incremental sequential-sum maps on a real ICP loop, on the CPU.

The d-bar chains of an ICP iteration (align_icp.cpp:113) differ from the
previous iteration's only where a correspondence changed.  This tool takes
the oracle's AlignIcp3d trace on a 640x480 pair of the bench stream,
rebuilds every iteration's correspondence stream (dst[nbr_i], d2_i), and runs
the host emulation of seqsum.hip (tests/cpp/seqsum_emu.cpp) over the
iterations twice: every map rebuilt from scratch, and incrementally (only
the maps of dirty blocks / groups / superblocks, the guesses of the last full
build).  It checks both against numpy's sequential float32 sums and prints
the maps built and the walk's superblock / group / leaf hits per iteration.

    python tools/seqsum_incr_sim.py [--iters 64 --pair 0]
"""
from __future__ import annotations

import argparse
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from oracle import oracle as O  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402
from seqsum_emu import binary  # noqa: E402


def streams(width, height, iters, pair):
    K = driver.intrinsics(width, height)
    sc = driver.SyntheticScene(0)
    da = sc.render(sc.trajectory(pair), K, noise_seed=pair)
    db = sc.render(sc.trajectory(pair + 1), K, noise_seed=pair + 1)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    dst = O.unproject(da, K4)
    src = O.unproject(db, K4)
    tree = O.KDTree(dst, 16)
    _, _, _, tr = O.align_icp(src, dst, iters, tree=tree, trace=True)
    out = np.zeros((iters, len(src), 4), np.float32)
    for it in range(iters):
        T = np.eye(4, dtype=np.float32) if it == 0 else tr["pose"][it - 1]
        idx, d2 = tree.query(O.transform_points(T, src))
        out[it, :, :3] = dst[idx]
        out[it, :, 3] = d2
    return out


def run(x, incremental):
    ns, n, _ = x.shape
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "in.f32"
        x.tofile(f)
        r = subprocess.run([str(binary()), str(f), str(n), "4", str(ns), str(int(incremental))],
                           capture_output=True, text=True, check=True)
    rows = [ln.split() for ln in r.stdout.splitlines() if ln.strip()]
    bits = np.array([int(t[0], 16) for t in rows], np.uint32).reshape(ns, 4)
    st = np.array([[int(v) for v in t[1:]] for t in rows], np.int64).reshape(ns, 4, -1)
    return bits, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--iters", type=int, default=64)
    ap.add_argument("--pair", type=int, default=0)
    ap.add_argument("--mode", type=int, default=2,
                    help="1: the guesses of the last full build; 2: a fresh front every "
                         "iteration, a clean block's map reused when its base is unchanged")
    a = ap.parse_args()
    x = streams(a.width, a.height, a.iters, a.pair)
    with np.errstate(all="ignore"):
        want = np.add.accumulate(np.concatenate([np.zeros((x.shape[0], 1, 4), np.float32), x], 1),
                                 axis=1, dtype=np.float32)[:, -1].view(np.uint32)
    full_b, full_s = run(x, False)
    inc_b, inc_s = run(x, a.mode)
    print(f"n {x.shape[1]}; full exact {np.array_equal(full_b, want)}; "
          f"incremental exact {np.array_equal(inc_b, want)}")
    print("it | chains x,y,z: leaves/groups/sbs built, walk sb hits/tries, group hits/tries, "
          "leaf hits/tries, serial blocks (full -> incremental)")
    for it in range(x.shape[0]):
        parts = []
        for c in range(3):
            f, g = full_s[it, c], inc_s[it, c]
            parts.append(f"{g[7]:5d}/{g[8]:4d}/{g[9]:2d} sb {f[1]}/{f[0]}->{g[1]}/{g[0]} "
                         f"g {f[3]}/{f[2]}->{g[3]}/{g[2]} l {f[5]}/{f[4]}->{g[5]}/{g[4]} "
                         f"s {f[6]}->{g[6]}")
        print(f"{it:3d} | " + " | ".join(parts))
    tot = lambda s, j: int(s[1:, :3, j].sum())  # noqa: E731
    print(f"iterations 1..: leaves built {tot(inc_s, 7)} vs {tot(full_s, 7)}, groups "
          f"{tot(inc_s, 8)} vs {tot(full_s, 8)}, superblocks {tot(inc_s, 9)} vs {tot(full_s, 9)}; "
          f"walk group tries {tot(inc_s, 2)} vs {tot(full_s, 2)}, leaf tries {tot(inc_s, 4)} vs "
          f"{tot(full_s, 4)}, serial blocks {tot(inc_s, 6)} vs {tot(full_s, 6)}")


if __name__ == "__main__":
    main()
