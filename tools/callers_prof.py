"""The reference callers' workload (rs_replay_app.cpp:229,246-251), as
bench.py's callers_workload leg: RemoveNans -> DownsampleVoxel(0.05) of both
clouds -> AlignIcp3d(curr_down, prev_down, 128) on host clouds, one pair at
a time, timed per pair and per phase; run under rocprofv3 --kernel-trace for
its per-iteration kernels (scripts/iter_profile_all.py).
  python tools/callers_prof.py [ref|fp64] [pairs]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "ref"
o = L.default_opts(sum_mode=L.RST_SUM_REF if mode == "ref" else L.RST_SUM_FP64)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
raw = [driver.unproject(sc.render(sc.trajectory(i), K, noise_seed=i), K, keep_invalid=True)
       for i in range(6)]


def timed(fn, *a, **kw):
    t0 = time.perf_counter()
    r = fn(*a, **kw)
    return r, 1000 * (time.perf_counter() - t0)


def pair(k):
    ph = []
    c, t = timed(A.RemoveNans, raw[k])
    ph.append(t)
    cur, t = timed(A.DownsampleVoxel, c, 0.05)
    ph.append(t)
    p, t = timed(A.RemoveNans, raw[k - 1])
    ph.append(t)
    prv, t = timed(A.DownsampleVoxel, p, 0.05)
    ph.append(t)
    T = np.eye(4, dtype=np.float32)
    _, da = timed(A.AlignIcp3d, cur, prv, 128, T, opts=o)
    return len(cur), ph, da


pair(1)
npairs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
for k in range(2, 2 + npairs):
    n, ph, da = pair(2 + (k - 2) % 4)
    print(f"pair {k}: n {n}  prepare {sum(ph):.2f} ms (nans / voxel / nans / voxel "
          f"{' / '.join(f'{x:.2f}' for x in ph)})  align {da:.2f} ms  total {sum(ph) + da:.2f} ms")
