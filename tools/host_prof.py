"""bench.py's host_api leg alone: AlignIcp3d(src, dst, 128, T) on host
640x480 clouds, one pair at a time, timed per pair; run under rocprofv3
--kernel-trace for its per-iteration kernels (scripts/iter_profile_all.py).
  python tools/host_prof.py [pairs]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

npairs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
clouds = [driver.unproject(sc.render(sc.trajectory(i), K, noise_seed=i), K) for i in range(npairs + 2)]
T = np.eye(4, dtype=np.float32)
A.AlignIcp3d(clouds[1], clouds[0], 128, T)  # (warm the context's pools)
for k in range(2, npairs + 2):
    T = np.eye(4, dtype=np.float32)
    t0 = time.perf_counter()
    A.AlignIcp3d(clouds[k], clouds[k - 1], 128, T)
    print(f"pair {k}: {1000 * (time.perf_counter() - t0):.2f} ms, {len(clouds[k])} points")
