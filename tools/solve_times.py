"""k_reduce_solve's two phases per iteration (the slab reduction and the
Kabsch solve; device clock, rst_debug_queue_trace) on a 640x480 pair, both
sum modes -- the solve is one thread's fp64 polar factor."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

lib = L.lib()
f = lib.rst_debug_queue_trace
f.restype, f.argtypes = C.c_int, [C.c_void_p, L.c_int32_p, C.c_int32]
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
da, db, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
bufs = [A.DeviceBuffer.from_array(x, ctx) for x in (da, db)]
t = A.Target.from_depth_device(bufs[0].ptr, K, 0, ctx)
s = A.Target.from_depth_device(bufs[1].ptr, K, 0, ctx)
for name, sm in (("fp64", L.RST_SUM_FP64), ("ref", L.RST_SUM_REF)):
    for rep in range(2):
        r = A.align_prepared(s, t, None, L.default_opts(max_iter=128, sum_mode=sm))
    q = np.zeros((256, 5), np.int32)
    f(ctx.handle, L.iptr(q), 256)
    red, sol = q[:128, 3] / 100.0, q[:128, 4] / 100.0  # 10 ns ticks -> us
    print(f"{name}: reduction {red.mean():.2f} us (max {red.max():.2f}), "
          f"solve {sol.mean():.2f} us (max {sol.max():.2f}) per iteration")
