"""Per-iteration anatomy of one 640x480 P2POINT pair (fp64 sums) with the
RST_DIAG library variant (RST_LIB=.../diag.so): points certified by
k_icp_nn, near / far queue lengths, queued entries the leaf adjacency
answered, ball-tile chunks, deep searches, and the kernel times (timing
pass on the same pair).

    RST_LIB=.../diag.so python tools/diag_fb.py [--host] [--bench-pair K] [--ref]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

lib = L.lib()
for name in ("rst_debug_queue_trace", "rst_debug_iter_diag"):
    f = getattr(lib, name)
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, L.c_int32_p, C.c_int32]
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
if "--bench-pair" in sys.argv:  # the bench stream's pair k: frames k-1 (target) and k (source)
    kp = int(sys.argv[sys.argv.index("--bench-pair") + 1])
    sc = driver.SyntheticScene(0)
    da = sc.render(sc.trajectory(kp - 1), K, noise_seed=kp - 1)
    db = sc.render(sc.trajectory(kp), K, noise_seed=kp)
else:
    da, db, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
if "--host" in sys.argv:  # clouds built from host points (no pixel grid)
    pa, pb = driver.unproject(da, K), driver.unproject(db, K)
    tgt = A.Target.build(pa, ctx)
    src = A.Target.build(pb, ctx)
else:  # frame targets prepared from depth on the device (the bench path)
    bufs = [A.DeviceBuffer.from_array(x, ctx) for x in (da, db)]
    tgt = A.Target.from_depth_device(bufs[0].ptr, K, 0, ctx)
    src = A.Target.from_depth_device(bufs[1].ptr, K, 0, ctx)
    pa, pb = np.zeros((len(tgt), 3)), np.zeros((len(src), 3))
opts = L.default_opts(max_iter=128, sum_mode=L.RST_SUM_REF if "--ref" in sys.argv else L.RST_SUM_FP64)
for rep in range(2):
    T = np.eye(4, dtype=np.float32)
    r = A.align_prepared_async(src, tgt, ctx, T, opts).wait()  # (second run: warm pools)
q = np.zeros((256, 5), np.int32)
lib.rst_debug_queue_trace(ctx.handle, L.iptr(q), 256)
d = np.zeros((256, 4), np.int32)
lib.rst_debug_iter_diag(ctx.handle, L.iptr(d), 256)
print("n", len(pb), "m", len(pa), "ok", r.ok)
print("  it  certified   nearQ    farQ  adj_exact  ball_chunks   pix_exact   deep  red_us solve_us")
for it in list(range(0, 20)) + [24, 32, 48, 64, 96, 127]:
    print(f"{it:4d} {q[it,1]:10d} {q[it,0]:7d} {d[it,0]:7d} {q[it,2]:10d} {d[it,1]:12d} "
          f"{d[it,2]:11d} {d[it,3]:6d} {q[it,3] / 100:7.2f} {q[it,4] / 100:8.2f}")
