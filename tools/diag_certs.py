"""Per-iteration anatomy of one 640x480 ICP pair on the GPU: fallback-queue
length, lanes answered by their certificate, lanes answered by the
adjacency search.  Needs a diagnostics build:
    RST_DEFINES=-DRST_DIAG=1 python -m realsensetracker_amd.build --lib --out lib/variants/diag.so
    RST_LIB=realsensetracker_amd/lib/variants/diag.so python tools/diag_certs.py"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from realsensetracker_amd import _lib as L, align as A, driver  # noqa: E402

lib = L.lib()
qt = lib.rst_debug_queue_trace
qt.restype = C.c_int
qt.argtypes = [C.c_void_p, L.c_int32_p, C.c_int32]
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
fa = A.Target.build(driver.unproject(sc.render(sc.trajectory(0), K, noise_seed=1), K), ctx)
fb = A.Target.build(driver.unproject(sc.render(sc.trajectory(1), K, noise_seed=2), K), ctx)
n = len(fb)
for sm in (L.RST_SUM_FP64,):
    r = A.align_prepared(fb, fa, None, L.default_opts(sum_mode=sm))
    q = np.zeros((256, 5), np.int32)
    qt(ctx.handle, L.iptr(q), 256)
    dg = np.zeros((256, 4), np.int32)
    dd = lib.rst_debug_iter_diag
    dd.restype = C.c_int
    dd.argtypes = [C.c_void_p, L.c_int32_p, C.c_int32]
    dd(ctx.handle, L.iptr(dg), 256)
    print(f"n={n} ok={r.ok}; iter: near-queue certified adj-exact (fractions of n), "
          "solve kernel: reduce us, solve us | far queue, ball chunks/wave, ball aborts, deep")
    for it in list(range(12)) + [16, 24, 32, 48, 64, 96, 127]:
        print(f"{it:4d} {q[it, 0] / n:8.4f} {q[it, 1] / n:8.4f} {q[it, 2] / n:8.4f}"
              f" {q[it, 3] * 0.01:7.2f} {q[it, 4] * 0.01:7.2f} | {dg[it, 0]:6d}"
              f" {dg[it, 1] / max(1, (n + 63) // 64):7.2f} {dg[it, 2]:6d} {dg[it, 3]:6d}")
