"""The sequential sums' walks inside the RST_SUM_REF loop, per iteration
(rst_debug_seq_walk_stats): superblock / group / leaf tries and hits,
serial blocks and walker clocks per chain, on a 640x480 frame pair."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

lib = L.lib()
for nm, args in (("rst_debug_enable_seq_trace", [C.c_void_p, C.c_int]),
                 ("rst_debug_seq_walk_stats", [C.c_void_p, C.c_void_p, C.c_int32])):
    getattr(lib, nm).restype, getattr(lib, nm).argtypes = C.c_int, args
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)  # the bench's stream (bench.py render_frames, seed 0, stride 1)
frames = [sc.render(sc.trajectory(i), K, noise_seed=i) for i in range(4)]
L.check(lib.rst_debug_enable_seq_trace(ctx.handle, 1), "trace")
tot_all = np.zeros((4, 8), np.int64)
for pi in range(3):
    bufs = [A.DeviceBuffer.from_array(x, ctx) for x in (frames[pi], frames[pi + 1])]
    t = A.Target.from_depth_device(bufs[0].ptr, K, 0, ctx)
    s = A.Target.from_depth_device(bufs[1].ptr, K, 0, ctx)
    r = A.align_prepared(s, t, None, L.default_opts(max_iter=128))
    st = np.zeros((128, 64), np.int32)
    L.check(lib.rst_debug_seq_walk_stats(ctx.handle, st.ctypes.data, 128), "stats")
    print(f"pair {pi}: per chain (x, y, z, cost) [sb tries/hits, group tries/hits, leaf tries/hits, serial, clocks]")
    for it in list(range(0, 8)) + [16, 32, 64, 127]:
        row = st[it, :32].reshape(4, 8)
        print(f"{it:4d}", " | ".join(f"{a[0]}/{a[1]} {a[2]}/{a[3]} {a[4]}/{a[5]} s{a[6]} c{a[7]}" for a in row))
    tot = st[:, :32].reshape(128, 4, 8).astype(np.int64).sum(0)
    tot_all += tot
    print("  sums per chain:", tot.tolist())
    print("  iterations with descents per chain:", [(st[:, c * 8] != st[:, c * 8 + 1]).sum() for c in range(4)])
    print("  map waits / descent phases, iterations 0-5:")
    for it in range(6):
        print(f"  {it:4d}", st[it, 33:37].tolist(), st[it, 57:63].tolist())
print("all pairs, per chain:", tot_all.tolist())
