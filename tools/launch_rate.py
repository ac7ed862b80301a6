"""Dispatch-rate probe: empty kernels per second over 1..32 streams
(rst_debug_launch_rate) -- the ceiling a chain of small dependent launches
per ICP iteration runs into when many frame pairs are in flight."""
import ctypes as C
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402

ctx = A.get_context(0)
f = L.lib().rst_debug_launch_rate
f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.POINTER(C.c_double)]
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"))
for blocks, threads in ((1, 64), (256, 256), (1024, 256)):
    for ns in (1, 4, 8, 16, 24, 32):
        r = C.c_double(0)
        L.check(f(ctx.handle, ns, max(200, 4000 // ns), blocks, threads, C.byref(r)), "launch_rate")
        print(f"blocks {blocks:5d} x {threads:4d}, streams {ns:3d}: {r.value / 1e3:8.1f} k kernels/s")
