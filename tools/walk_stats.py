"""The sequential sums' walks inside the RST_SUM_REF loop, per iteration
(rst_debug_seq_walk_stats): superblock / group / leaf tries and hits,
serial blocks and walker clocks per chain, on a 640x480 frame pair.

    python tools/walk_stats.py [--first 0 --pairs 3 --brief]
(--brief: one line per pair -- descents, serial blocks, the slowest chain's
walker clocks summed over the iterations)"""
import argparse
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
ap = argparse.ArgumentParser()
ap.add_argument("--first", type=int, default=0)
ap.add_argument("--pairs", type=int, default=3)
ap.add_argument("--brief", action="store_true")
a = ap.parse_args()
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)  # the bench's stream (bench.py render_frames, seed 0, stride 1)
frames = {i: sc.render(sc.trajectory(i), K, noise_seed=i) for i in range(a.first, a.first + a.pairs + 1)}
L.check(lib.rst_debug_enable_seq_trace(ctx.handle, 1), "trace")
tot_all = np.zeros((4, 8), np.int64)
for pi in range(a.first, a.first + a.pairs):
    bufs = [A.DeviceBuffer.from_array(x, ctx) for x in (frames[pi], frames[pi + 1])]
    t = A.Target.from_depth_device(bufs[0].ptr, K, 0, ctx)
    s = A.Target.from_depth_device(bufs[1].ptr, K, 0, ctx)
    r = A.align_prepared(s, t, None, L.default_opts(max_iter=128))
    st = np.zeros((128, 64), np.int32)
    L.check(lib.rst_debug_seq_walk_stats(ctx.handle, st.ctypes.data, 128), "stats")
    tot = st[:, :32].reshape(128, 4, 8).astype(np.int64)
    if a.brief:
        desc = (tot[:, :, 0] != tot[:, :, 1]).sum(0)
        print(f"pair {pi}: iterations with descents per chain {desc.tolist()}, group tries "
              f"{tot[:, :, 2].sum(0).tolist()}, leaf tries {tot[:, :, 4].sum(0).tolist()}, serial "
              f"{tot[:, :, 6].sum(0).tolist()}, slowest chain clocks per iteration: mean "
              f"{tot[:, :, 7].max(1).mean():.0f}, iterations 0-7 {tot[:8, :, 7].max(1).tolist()}", flush=True)
        rt = st[:, [37, 38, 39, 56]].astype(np.float64)  # 100 MHz ticks of the same walks
        clk = tot[:, :, 7].astype(np.float64)
        ok = rt > 0
        print(f"  walker clock rate {np.median(clk[ok] / rt[ok]) * 0.1:.2f} GHz (s_memtime / s_memrealtime)")
        tp = st[:, 40:52].reshape(-1, 2, 6).astype(np.int64).sum(0)
        for c in range(2):
            print(f"  chain {c} descents, clocks over the align: group load {tp[c, 0]}, group steps {tp[c, 1]}, "
                  f"leaf load {tp[c, 2]}, leaf steps {tp[c, 3]}, own adds {tp[c, 4]}, whole {tp[c, 5]} "
                  f"(of walks {int(tot[:, c, 7].sum())})")
        tot_all += tot.sum(0)
        for b in bufs:
            b.free()
        s.free()
        t.free()
        continue
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
