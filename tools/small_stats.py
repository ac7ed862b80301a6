"""Phase clocks and walk counts of k_sq_small (the one-workgroup-per-chain
sequential sums, seqsum.hip) on callers-like chains: python tools/small_stats.py"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

f = L.lib().rst_debug_seq_sum
f.restype = C.c_int
f.argtypes = [C.c_void_p, L.c_float_p, C.c_int64, C.c_int, C.c_int, L.c_float_p, C.POINTER(C.c_float),
              C.c_void_p]
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
da, db, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
cloud = A.DownsampleVoxel(A.RemoveNans(driver.unproject(da, K)), 0.05)
rng = np.random.default_rng(1)
cases = {"callers_cloud": np.concatenate([cloud, (cloud * cloud).sum(1, keepdims=True)], 1),
         "uniform_1024": rng.standard_normal((1024, 4)),
         "uniform_15k": rng.standard_normal((15239, 4)),
         "positive_15k": rng.uniform(0.3, 5.0, (15239, 4))}
for name, x in cases.items():
    x = np.ascontiguousarray(x, np.float32)
    for code in (4, 2):
        out = np.zeros(4, np.float32)
        ms = C.c_float(0)
        st = np.zeros(64, np.int32)
        L.check(f(ctx.handle, L.fptr(x), len(x), code, 10, L.fptr(out), C.byref(ms), st.ctypes.data), "seq")
        if code == 4:
            print(f"{name} n={len(x)}: small {ms.value * 1e3:.1f} us; chain 0 phase clocks "
                  f"{st[:6].tolist()}; groups tried/hit {st[8]}/{st[9]} of {st[13]}, leaves "
                  f"tried/hit {st[10]}/{st[11]}, serial blocks {st[12]}")
        else:
            print(f"   maps {ms.value * 1e3:.1f} us")
