"""Kernels at once from independent streams vs the kernel's duration
(rst_debug_kernel_overlap; 1 block x 64 threads, no LDS): a dispatch-rate
ceiling shows as overlap ~ rate x duration, a cap on concurrent kernels as
a plateau whatever the duration."""
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
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
blocks = int(os.environ.get("OV_BLOCKS", "1"))
for spin in (10, 40, 160, 640):
    row = []
    for ns in (1, 4, 8, 16, 24, 32):
        nl = max(4, int(64000 / spin / ns))  # ~64 ms of busy time per stream set
        best = 0.0
        for _ in range(2):
            r = C.c_double(0)
            L.check(f(ctx.handle, ns, nl, blocks, 64, spin, 0, C.byref(r)), "overlap")
            best = max(best, r.value)
        row.append(f"{ns}:{best:5.2f}")
    print(f"spin {spin:4d} us, {blocks} blocks -> kernels at once " + " ".join(row), flush=True)
