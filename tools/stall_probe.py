"""Where the callers' workload's first host call after an AlignIcp3d waits
(profiles/r05_callers_prof.txt: the first RemoveNans of each pair 20-28 ms,
the second 0.8 ms): after each align, (a) a 10-point RemoveNans, (b) a
30 ms sleep, or (c) nothing, then the full-frame RemoveNans, timed.
  python tools/stall_probe.py"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
raw = [driver.unproject(sc.render(sc.trajectory(i), K, noise_seed=i), K, keep_invalid=True)
       for i in range(3)]
cur = A.DownsampleVoxel(A.RemoveNans(raw[1]), 0.05)
prv = A.DownsampleVoxel(A.RemoveNans(raw[0]), 0.05)
tiny = raw[2][:10].copy()


def ms(fn, *a):
    t0 = time.perf_counter()
    fn(*a)
    return 1000 * (time.perf_counter() - t0)


for rep in range(3):
    for mode in ("none", "tiny", "sleep", "align_fp64_none"):
        T = np.eye(4, dtype=np.float32)
        if mode == "align_fp64_none":
            from realsensetracker_amd import _lib as L
            ta = ms(lambda: A.AlignIcp3d(cur, prv, 128, T, opts=L.default_opts(sum_mode=L.RST_SUM_FP64)))
        else:
            ta = ms(A.AlignIcp3d, cur, prv, 128, T)
        pre = ""
        if mode == "tiny":
            pre = f"tiny {ms(A.RemoveNans, tiny):.2f} "
        elif mode == "sleep":
            time.sleep(0.03)
        t1 = ms(A.RemoveNans, raw[2])
        t2 = ms(A.RemoveNans, raw[2])
        print(f"rep {rep} {mode:16s} align {ta:6.2f}  {pre}nans#1 {t1:6.2f}  nans#2 {t2:5.2f} ms", flush=True)
