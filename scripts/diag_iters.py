"""GPU AlignIcp3d vs the fp64-sum oracle after 1..N iterations (golden pair)."""
import ctypes as C
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_golden
from oracle import oracle as O
from posemetric import pose_err
from realsensetracker_amd import _lib as L, align as A

lib = L.lib()
qt = lib.rst_debug_queue_trace
qt.restype = C.c_int
qt.argtypes = [C.c_void_p, L.c_int32_p, C.c_int32]
ctx = A.get_context(0)
g = load_golden(sys.argv[1] if len(sys.argv) > 1 else "pair_80x60_s0")
t = A.Target.build(g["dst"], ctx)
for it in (1, 2, 3, 4, 6, 8, 16, 32):
    T = np.eye(4, dtype=np.float32)
    A.AlignIcp3d(g["src"], g["dst"], t, it, T)
    _, To, _, _ = O.align_icp(g["src"], g["dst"], it, sum_mode=1)
    q = np.zeros((256, 5), np.int32)
    qt(ctx.handle, L.iptr(q), 256)
    print(it, "err", pose_err(T, To), "listed/rebuild/fallback per iter:",
          [(int(q[k, 1]), int(q[k, 2]), int(q[k, 0])) for k in range(it)][:8])
