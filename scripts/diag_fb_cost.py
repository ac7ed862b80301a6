"""Cycle cost of the fallback search strategies on far / near queries."""
import ctypes as C
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
from oracle import oracle as O
from realsensetracker_amd import _lib as L, align as A, driver

ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(3)
da, db, _ = driver.make_pair(sc, K, seed=31)
pa = driver.unproject(da, K, ctx=ctx); pb = driver.unproject(db, K, ctx=ctx)
t = A.Target.build(pa, ctx); tree = O.KDTree(pa)
f = L.lib().rst_debug_query_nn_fallback
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_void_p, L.c_float_p, C.c_int64, L.c_int32_p, C.c_int, L.c_int32_p, L.c_float_p, L.c_int32_p]
rng = np.random.default_rng(0)
for lo, hi in ((1e-3, 3e-3), (3e-3, 1e-2), (1e-2, 3e-2), (3e-2, 0.1), (0.1, 0.5)):
    sel = rng.choice(len(pb), 2000, replace=False)
    off = rng.normal(size=(2000, 3)).astype(np.float32)
    off *= rng.uniform(lo, hi, 2000).astype(np.float32)[:, None] / np.linalg.norm(off, axis=1, keepdims=True)
    q = np.ascontiguousarray(pb[sel] + off, np.float32)
    warm, _ = tree.query(pb[sel])
    warm = warm.astype(np.int32)
    line = [f"|off| {lo*1e3:5.1f}-{hi*1e3:6.1f} mm:"]
    for mode in (0, 2, 3, 23):
        idx = np.zeros(2000, np.int32); d2 = np.zeros(2000, np.float32); path = np.zeros(2000, np.int32)
        L.check(f(ctx.handle, t.handle, L.fptr(q), 2000, L.iptr(warm), mode, L.iptr(idx), L.fptr(d2), L.iptr(path)), "fb")
        cyc = (path >> 4) * 16
        how = path & 15
        line.append(f"mode {mode}: med {np.median(cyc)/1e3:6.1f}k p99 {np.percentile(cyc,99)/1e3:6.1f}k max {cyc.max()/1e3:6.1f}k cyc, paths {np.bincount(how, minlength=4)[[0,2,3]].tolist()}")
    print("\n   ".join(line))
