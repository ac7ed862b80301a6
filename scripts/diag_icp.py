"""Per-iteration picture of one 640x480 AlignIcp3d on the GPU: fallback
queue length per iteration, pose vs the oracle-free ground truth, timing."""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402


def main():
    W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (640, 480)
    lib = L.lib()
    qt = lib.rst_debug_queue_trace
    qt.restype = C.c_int
    qt.argtypes = [C.c_void_p, L.c_int32_p, C.c_int32]
    ctx = A.get_context(0)
    K = driver.intrinsics(W, H)
    sc = driver.SyntheticScene(0)
    for pair in range(2):
        da = sc.render(sc.trajectory(pair), K, noise_seed=1 + pair)
        db = sc.render(sc.trajectory(pair + 1), K, noise_seed=2 + pair)
        pa = driver.unproject(da, K)
        pb = driver.unproject(db, K)
        t0 = time.perf_counter()
        ta = A.Target.build(pa, ctx)
        ctx.synchronize()
        t1 = time.perf_counter()
        tb = A.Target.build(pb, ctx)
        for mode, it in [(L.RST_P2POINT_REF, 128), (L.RST_P2PLANE, 30)]:
            if mode == L.RST_P2PLANE:
                ta.compute_normals(16)
            ctx.synchronize()
            t2 = time.perf_counter()
            r = A.align_prepared(tb, ta, None, L.default_opts(mode=mode, max_iter=it))
            t3 = time.perf_counter()
            q = np.zeros((256, 5), np.int32)
            qt(ctx.handle, L.iptr(q), 256)
            print(f"pair {pair} mode {mode}: n={len(pb)} build {1e3*(t1-t0):.2f} ms  align "
                  f"{1e3*(t3-t2):.2f} ms  iters {r.iterations} ok {r.ok}")
            print("  slow queue per iteration:", " ".join(str(x) for x in q[:r.iterations, 0]))
            print("  answered by candidate list:", " ".join(str(x) for x in q[:r.iterations, 1]))
            print("  lists rebuilt (slow kernel):", " ".join(str(x) for x in q[:r.iterations, 2]))
            print("  solve kernel: reduce / solve (x10 ns):", " ".join(f"{a}/{b}" for a, b in q[:min(r.iterations, 24), 3:5]))


if __name__ == "__main__":
    main()
