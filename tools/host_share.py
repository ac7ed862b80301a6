"""Where the host thread of the REF value leg spends its time: frame
preparation (unprojection + index build, enqueued), the align's enqueue
(icp_launch: 128 iterations x the loop's kernels) and waiting for a pair
to finish.  If the enqueue takes most of the wall time, the host's launch
path -- not the GPU -- bounds the throughput.

    GPU_MAX_HW_QUEUES=24 python tools/host_share.py [--inflight 24 --steps 48 --graphs]
"""
import argparse
import sys
import time
from collections import deque
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--inflight", type=int, default=24)
ap.add_argument("--steps", type=int, default=48)
ap.add_argument("--graphs", action="store_true")
ap.add_argument("--threads", type=int, default=0, help="enqueue aligns from a pool of this many threads")
a = ap.parse_args()
import ctypes as C  # noqa: E402

K = driver.intrinsics(640, 480)
frames = bench.render_frames(0, 64, K, 1)
hip = C.CDLL("libamdhip64.so")
d_depth = []
for f in frames:
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), C.c_size_t(2 * 640 * 480)) == 0
    assert hip.hipMemcpy(p, f.ctypes.data_as(C.c_void_p), C.c_size_t(2 * 640 * 480), 1) == 0
    d_depth.append(p)
opts = L.default_opts(max_iter=128, sum_mode=L.RST_SUM_REF)
pctx = A.Context(0)
ctxs = [A.Context(0) for _ in range(a.inflight)]
if a.graphs:
    for c in ctxs:
        c.enable_graphs(True)
pool = None
if a.threads > 0:
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(a.threads)


def run(nsteps, t):
    pending = deque()
    prev = A.Target.from_depth_device(d_depth[0].value, K, 0, pctx)
    for s in range(nsteps):
        t0 = time.perf_counter()
        cur = A.Target.from_depth_device(d_depth[bench.pingpong(s + 1, 64)].value, K, 0, pctx)
        t1 = time.perf_counter()
        if len(pending) == len(ctxs):
            fut, tg, sr = pending.popleft()
            pa = fut.result() if pool else fut
            pa.wait()
            tg.free()
        t2 = time.perf_counter()
        c = ctxs[s % len(ctxs)]
        if pool:
            fut = pool.submit(A.align_prepared_async, cur, prev, c, None, opts)
        else:
            fut = A.align_prepared_async(cur, prev, c, None, opts)
        t3 = time.perf_counter()
        pending.append((fut, prev, cur))
        prev = cur
        t["prep"] += t1 - t0
        t["wait"] += t2 - t1
        t["enqueue"] += t3 - t2
    while pending:
        fut, tg, sr = pending.popleft()
        pa = fut.result() if pool else fut
        pa.wait()
        tg.free()
    prev.free()


run(len(ctxs) + 2, {"prep": 0, "wait": 0, "enqueue": 0})
t = {"prep": 0.0, "wait": 0.0, "enqueue": 0.0}
pctx.synchronize()
T0 = time.perf_counter()
run(a.steps, t)
for c in ctxs:
    c.synchronize()
T = time.perf_counter() - T0
print(f"inflight {a.inflight} graphs {a.graphs} threads {a.threads}: {a.steps * 128 / T:.0f} ICP it/s; "
      f"wall {T * 1e3:.0f} ms: prep {t['prep'] * 1e3:.0f} ms, enqueue {t['enqueue'] * 1e3:.0f} ms "
      f"({t['enqueue'] / a.steps * 1e3:.2f} ms per align), wait {t['wait'] * 1e3:.0f} ms", flush=True)
