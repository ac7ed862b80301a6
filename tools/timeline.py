"""The REF loop's kernels under load, from the device's own clock (no
tracer): a RST_TIMELINE build records, per iteration and loop kernel, the
earliest wave start and the latest wave end of every align.  This runs the
value leg (24 frame pairs in flight, one context each) and reads the last
align of every context -- aligns that ran side by side -- for the kernels'
durations under load, the gaps between one pair's consecutive kernels
(dispatch and queueing), and how many kernels ran at once.

    RST_DEFINES=-DRST_TIMELINE=1 python -m realsensetracker_amd.build --lib \\
        --out $PWD/realsensetracker_amd/lib/variants/timeline.so
    RST_LIB=realsensetracker_amd/lib/variants/timeline.so GPU_MAX_HW_QUEUES=24 \\
        python tools/timeline.py [--inflight 24]
"""
import argparse
import ctypes as C
import sys
from collections import deque
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

NAMES = ["nn", "fb", "sq_tot", "sq_front", "sq_build", "sq_walk", "cov_ref", "solve"]
ap = argparse.ArgumentParser()
ap.add_argument("--inflight", type=int, default=24)
ap.add_argument("--steps", type=int, default=48)
a = ap.parse_args()

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
fn = L.lib().rst_debug_timeline
fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32, C.POINTER(C.c_int32)]

pending = deque()
prev = A.Target.from_depth_device(d_depth[0].value, K, 0, pctx)
for s in range(a.steps):
    cur = A.Target.from_depth_device(d_depth[bench.pingpong(s + 1, 64)].value, K, 0, pctx)
    if len(pending) == len(ctxs):
        pa, tg = pending.popleft()
        pa.wait()
        tg.free()
    pending.append((A.align_prepared_async(cur, prev, ctxs[s % len(ctxs)], None, opts), prev))
    prev = cur
while pending:
    pa, tg = pending.popleft()
    pa.wait()
    tg.free()
prev.free()

tls = []
for c in ctxs:
    buf = (C.c_uint64 * (256 * 8 * 2))()
    it = C.c_int32(0)
    L.check(fn(c.handle, buf, 256 * 8 * 2, C.byref(it)), "rst_debug_timeline")
    t = np.frombuffer(buf, np.uint64).reshape(256, 8, 2)[:it.value].astype(np.float64) * 10.0  # ns
    tls.append(t)
t0 = min(t[0, 0, 0] for t in tls)
ivals = []  # (start, end, kernel) over every context's last align
for t in tls:
    for k in range(8):
        for i in range(len(t)):
            if t[i, k, 1] > 0:
                ivals.append((t[i, k, 0] - t0, t[i, k, 1] - t0, k))
# the window where most contexts' last aligns run (the middle half of their span)
st0 = sorted(t[0, 0, 0] - t0 for t in tls)
en0 = sorted(t[-1, 7, 1] - t0 for t in tls)
lo, hi = st0[-1] if len(tls) == 1 else st0[len(tls) // 2], en0[0] if len(tls) == 1 else en0[len(tls) // 2]
if hi <= lo:
    lo, hi = min(st0), max(en0)
print(f"{len(tls)} aligns side by side; common window {lo / 1e3:.0f} .. {hi / 1e3:.0f} us")
if hi > lo:
    pts = sorted([(max(s, lo), 1) for s, e, _ in ivals if e > lo and s < hi] +
                 [(min(e, hi), -1) for s, e, _ in ivals if e > lo and s < hi])
    cur, last, hist = 0, lo, {}
    for tt, d in pts:
        hist[cur] = hist.get(cur, 0.0) + (tt - last)
        cur += d
        last = tt
    w = hi - lo
    mean = sum(c * v for c, v in hist.items()) / w
    print(f"kernels running at once: mean {mean:.2f}; share of time " +
          ", ".join(f"{c}: {100 * v / w:.1f}%" for c, v in sorted(hist.items()) if v / w > 0.005))
    it_time = np.mean([(t[-1, 7, 1] - t[8, 0, 0]) / (len(t) - 8) for t in tls]) / 1e3
    print(f"one pair's iteration under load: {it_time:.1f} us (iterations 8..end); "
          f"{len(tls) / it_time * 1e6:.0f} ICP it/s from {len(tls)} pairs")
dur = np.concatenate([t[8:, :, 1] - t[8:, :, 0] for t in tls]) / 1e3
gaps = []
for t in tls:
    seq = t[8:].reshape(-1, 2)  # kernel order within an iteration, iterations in order
    gaps.append((seq[1:, 0] - seq[:-1, 1]).reshape(-1))
g = np.concatenate(gaps) / 1e3
gk = np.concatenate([x.reshape(-1, 1) for x in gaps]).reshape(-1)
print(f"{'kernel':<10}{'mean us':>9}{'p50':>8}{'p90':>8}{'  gap before (mean / p50 / p90 us)':>36}")
for k in range(8):
    d = dur[:, k]
    gb = np.concatenate([(t[8:, k, 0] - (t[8:, k - 1, 1] if k > 0 else np.concatenate([[t[7, 7, 1]], t[8:-1, 7, 1]])))
                         for t in tls]) / 1e3
    print(f"{NAMES[k]:<10}{d.mean():9.1f}{np.median(d):8.1f}{np.percentile(d, 90):8.1f}"
          f"{gb.mean():14.1f}{np.median(gb):8.1f}{np.percentile(gb, 90):8.1f}")
print(f"per iteration: kernels {dur.sum(1).mean():.1f} us, gaps {g.mean() * 8:.1f} us")
