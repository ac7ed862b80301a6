"""How many kernels from independent streams the GPU runs at once
(rst_debug_kernel_overlap): kernels whose waves only wait on the clock, so
nothing but the dispatch path limits their overlap.  The REF value leg keeps
24 frame pairs in flight on 24 streams; this is the ceiling their kernels
meet.

    GPU_MAX_HW_QUEUES=24 python tools/kernel_overlap.py
"""
import ctypes as C
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402

ctx = A.get_context(0)
f = L.lib().rst_debug_kernel_overlap
f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.POINTER(C.c_double)]
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"))
for blocks, threads, lds in ((1, 64, 0), (64, 256, 0), (256, 512, 0), (1, 64, 90 * 1024), (219, 512, 90 * 1024)):
    for spin in (20, 5):
        row = []
        for ns in (1, 2, 4, 8, 16, 24, 32):
            r = C.c_double(0)
            L.check(f(ctx.handle, ns, max(50, 1600 // ns), blocks, threads, spin, lds, C.byref(r)), "overlap")
            row.append(f"{ns}:{r.value:5.2f}")
        print(f"blocks {blocks:4d} x {threads:4d} lds {lds // 1024:3d} KB spin {spin:2d} us -> kernels at once "
              + " ".join(row), flush=True)
