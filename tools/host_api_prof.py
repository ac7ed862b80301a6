"""The reference-shaped host API, AlignIcp3d(src, dst, 128, T) on host
clouds of the bench's stream (as bench.py's host_api leg), timed per pair;
run under rocprofv3 --kernel-trace for its per-iteration kernels
(scripts/iter_profile_all.py) and the time outside them."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
frames = [sc.render(sc.trajectory(i), K, noise_seed=i) for i in range(4)]
clouds = [driver.unproject(f, K) for f in frames]
T = np.eye(4, dtype=np.float32)
A.AlignIcp3d(clouds[1], clouds[0], 128, T)
for k in range(1, 4):
    T = np.eye(4, dtype=np.float32)
    t0 = time.perf_counter()
    A.AlignIcp3d(clouds[k], clouds[k - 1], 128, T)
    print(f"pair {k}: {1000 * (time.perf_counter() - t0):.2f} ms")
