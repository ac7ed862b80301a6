"""The reference callers' workload (rs_replay_app.cpp:229,246-251), as
bench.py's callers_workload leg: RemoveNans -> DownsampleVoxel(0.05) of both
clouds -> AlignIcp3d(curr_down, prev_down, 128) on host clouds, one pair at
a time, timed per pair and per phase; run under rocprofv3 --kernel-trace for
its per-iteration kernels (scripts/iter_profile_all.py).
  python tools/callers_prof.py [ref|fp64]"""
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


def pair(k):
    t0 = time.perf_counter()
    cur = A.DownsampleVoxel(A.RemoveNans(raw[k]), 0.05)
    prv = A.DownsampleVoxel(A.RemoveNans(raw[k - 1]), 0.05)
    t1 = time.perf_counter()
    T = np.eye(4, dtype=np.float32)
    A.AlignIcp3d(cur, prv, 128, T, opts=o)
    t2 = time.perf_counter()
    return len(cur), 1000 * (t1 - t0), 1000 * (t2 - t1)


pair(1)
for k in range(2, 6):
    n, dp, da = pair(k)
    print(f"pair {k}: n {n}  prepare {dp:.2f} ms  align {da:.2f} ms  total {dp + da:.2f} ms")
