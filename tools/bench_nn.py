"""Cold exact-NN strategies on one 640x480 frame pair (iteration 0 of an
ICP pair: source at the identity pose against the previous frame):
lane-per-query top-down walk vs the wave-cooperative region search.
    python tools/bench_nn.py"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from realsensetracker_amd import _lib as L, align as A, driver  # noqa: E402

lib = L.lib()
f = lib.rst_debug_query_nn_warm_stats
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_void_p, L.c_float_p, C.c_int64, L.c_int32_p, L.c_int32_p,
              L.c_float_p, L.c_int32_p]
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
pa = driver.unproject(sc.render(sc.trajectory(0), K, noise_seed=1), K)
pb = driver.unproject(sc.render(sc.trajectory(1), K, noise_seed=2), K)
t = A.Target.build(pa, ctx)
src = A.Target.build(pb, ctx)


def morton_order(p):
    lo = p.min(0)
    ext = (p.max(0) - lo).max()
    qv = np.clip(((p - lo) * (1023.0 / ext)).astype(np.int64), 0, 1023)
    code = np.zeros(len(p), np.int64)
    for b in range(10):
        for a in range(3):
            code |= ((qv[:, a] >> b) & 1) << (3 * b + (2 - a))
    return np.argsort(code, kind="stable")


q = np.ascontiguousarray(pb)
qm = np.ascontiguousarray(pb[morton_order(pb)])
for rep in range(3):
    t0 = time.perf_counter()
    gi, gd = t.query(q)
    t1 = time.perf_counter()
    print(f"lane top-down walk (incl. upload/readback): {1e3 * (t1 - t0):.2f} ms")
nw = (len(q) + 63) // 64
stats = np.zeros(8 * nw, np.int32)
idx = np.zeros(len(q), np.int32)
d2 = np.zeros(len(q), np.float32)
for name, qq in (("input order", q), ("Morton order", qm)):
    for rep in range(3):
        L.check(f(ctx.handle, t.handle, L.fptr(qq), len(qq), None, L.iptr(idx), L.fptr(d2),
                  L.iptr(stats)), "warm")
        ms, _ = ctx.last_kernel_time()
        gi2, _ = t.query(qq) if rep == 0 else (gi2, None)
        print(f"wave region search, cold, {name}: kernel {ms:.3f} ms; exact={np.array_equal(idx, gi2)}")
