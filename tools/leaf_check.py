"""Leaf sizes of frame targets built like bench.py's stream (diagnostic):
every leaf must hold <= 16 points (rst_bvh.hpp leaf_cut).
  python tools/leaf_check.py"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from realsensetracker_amd import _lib as L, align as A, driver  # noqa: E402

lib = L.lib()
f = lib.rst_debug_target_leaves
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_int32),
              C.POINTER(C.c_int32)]
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
ctx = A.Context(0)
frames = [sc.render(sc.trajectory(i), K, noise_seed=i) for i in range(6)]
bufs = [A.DeviceBuffer.from_array(d, ctx) for d in frames]
bad = 0
for rep in range(3):
    for k, b in enumerate(bufs):
        for nk in (0, -2):
            t = A.Target.from_depth_device(b.ptr, K, nk, ctx)
            nl = C.c_int32()
            f(ctx.handle, t.handle, None, 0, None, C.byref(nl))
            ls = np.zeros(nl.value + 1, np.int32)
            L.check(f(ctx.handle, t.handle, ls.ctypes.data_as(C.POINTER(C.c_int32)), len(ls),
                      None, C.byref(nl)), "leaves")
            sz = np.diff(ls)
            m = len(t)
            if sz.max() > 16 or sz.min() < 0 or ls[-1] != m or ls[0] != 0:
                bad += 1
                j = int(np.argmax(sz))
                print(f"rep {rep} frame {k} nk {nk}: m={m} nl={nl.value} max leaf {sz.max()} at {j} "
                      f"(begin {ls[j]}), min {sz.min()}, lstart[0]={ls[0]} lstart[nl]={ls[-1]}")
            t.free()
print("bad targets:", bad)
