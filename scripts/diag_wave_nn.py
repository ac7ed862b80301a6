"""Diagnostics of the wave-cooperative NN search on a 640x480 frame pair:
per-wave staging / scan statistics for several warm-start situations."""
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


def spread(v):
    v = v.astype(np.uint32) & 0x3FF
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    v = (v | (v << 2)) & 0x09249249
    return v


def morton_sort(p):
    lo = p.min(0)
    ext = (p.max(0) - lo).max()
    q = np.clip((p - lo) * (1023.0 / ext), 0, 1023).astype(np.uint32)
    code = (spread(q[:, 0]) << 2) | (spread(q[:, 1]) << 1) | spread(q[:, 2])
    return p[np.argsort(code, kind="stable")]


def main():
    lib = L.lib()
    f = lib.rst_debug_query_nn_warm_stats
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_void_p, L.c_float_p, C.c_int64, L.c_int32_p, L.c_int32_p,
                  L.c_float_p, L.c_int32_p]
    ctx = A.get_context(0)
    W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (640, 480)
    K = driver.intrinsics(W, H)
    sc = driver.SyntheticScene(0)
    da = sc.render(sc.trajectory(0), K, noise_seed=1)
    db = sc.render(sc.trajectory(1), K, noise_seed=2)
    pa = driver.unproject(da, K)
    pb = morton_sort(driver.unproject(db, K))
    ta = A.Target.build(pa, ctx)
    tb = A.Target.build(pb, ctx)
    r = A.align_prepared(tb, ta)
    T = r.pose
    print("n", len(pb), "m", len(pa), "icp ok", r.ok, "iters", r.iterations)

    def stats_for(Tq, warm, label):
        q = (pb @ T[:3, :3].T.astype(np.float32) + T[:3, 3].astype(np.float32)).astype(np.float32) \
            if Tq is None else (pb @ Tq[:3, :3].T + Tq[:3, 3]).astype(np.float32)
        n = len(q)
        idx = np.zeros(n, np.int32)
        d2 = np.zeros(n, np.float32)
        st = np.zeros((n + 63) // 64 * 8, np.int32)
        w = None if warm is None else np.ascontiguousarray(warm, np.int32)
        t0 = time.perf_counter()
        L.check(f(ctx.handle, ta.handle, L.fptr(q), n, L.iptr(w) if w is not None else None,
                  L.iptr(idx), L.fptr(d2), L.iptr(st)), "stats")
        dt = time.perf_counter() - t0
        st = st.reshape(-1, 8)
        names = ["rounds", "nodes", "staged", "scanned", "wave_us", "active", "nobound", "ext_um"]
        st = st.astype(np.float64)
        st[:, 4] *= 0.01
        print(f"--- {label}: wall {dt*1e3:.1f} ms (incl. upload), kernel {ctx.last_kernel_time()[0]*1e3:.1f} us")
        for k, nm in enumerate(names):
            v = st[:, k].astype(np.float64)
            print(f"  {nm:8s} mean {v.mean():10.1f}  p50 {np.percentile(v,50):10.1f}  "
                  f"p90 {np.percentile(v,90):10.1f}  p99 {np.percentile(v,99):10.1f}  max {v.max():10.0f}")
        print("  capped waves:", int((st[:, 5] < 0).sum()), "of", len(st))
        slow = np.argsort(st[:, 4])[-5:]
        for w in slow:
            print("   slow wave", w, " ".join(f"{nm}={st[w,k]:.0f}" for k, nm in enumerate(names)))
        return idx, d2, q

    idx0, _, q0 = stats_for(np.eye(4, dtype=np.float32), None, "identity pose, cold")
    idx1, d21, q1 = stats_for(None, None, "converged pose, cold")
    stats_for(None, idx1, "converged pose, warm = exact answer")
    stats_for(None, idx0, "converged pose, warm = identity-pose NN")
    # where are the large regions? distance of the answer
    d = np.sqrt(d21)
    print("converged NN distance mm: p50 %.2f p90 %.2f p99 %.2f max %.1f" % tuple(
        np.percentile(d, [50, 90, 99]).tolist() + [d.max()]))
    per_wave_max = np.array([d[i:i + 64].max() for i in range(0, len(d), 64)]) * 1e3
    print("per-wave max NN distance mm: p50 %.2f p90 %.2f p99 %.2f" % tuple(np.percentile(per_wave_max, [50, 90, 99])))


if __name__ == "__main__":
    main()
