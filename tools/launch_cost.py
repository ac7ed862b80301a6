"""Host cost of enqueueing one batched align (rst_icp_align_batch_async:
128 iterations x ~10 launches) against its GPU time, on the bench's frames.
    python tools/launch_cost.py [pairs]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 12
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
tg = []
bufs = []
for i in range(nb + 1):
    d = A.DeviceBuffer.from_array(sc.render(sc.trajectory(i), K, noise_seed=i), ctx)
    bufs.append(d)
    tg.append(A.Target.from_depth_device(d.ptr, K, 0, ctx))
ctx.synchronize()
for rep in range(4):
    t0 = time.perf_counter()
    p = A.align_batch_async(tg[1:], tg[:-1], ctx)
    t1 = time.perf_counter()
    r = p.wait()
    t2 = time.perf_counter()
    print(f"rep {rep}: enqueue {1000 * (t1 - t0):.2f} ms, then wait {1000 * (t2 - t1):.2f} ms, ok {sum(x.ok for x in r)}/{nb}")
