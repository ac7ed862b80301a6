"""k_icp_nn's wave latencies in one iteration (RST_NN_CLK_ITER, default
64) of a 640x480 REF pair, from a diagnostics build:
    RST_DEFINES=-DRST_NN_CLK=1 python -m realsensetracker_amd.build --lib --out $PWD/realsensetracker_amd/lib/variants/nnclk.so
    RST_LIB=realsensetracker_amd/lib/variants/nnclk.so python tools/nn_clock.py
Per wave: start / end (realtime, 10 ns), shader clocks to the certificate
test, in the pixel search, in total."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

lib = L.lib()
f = lib.rst_debug_slab
f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]
ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
fr = [sc.render(sc.trajectory(i), K, noise_seed=i) for i in range(2)]
bufs = [A.DeviceBuffer.from_array(x, ctx) for x in fr]
t = A.Target.from_depth_device(bufs[0].ptr, K, 0, ctx)
s = A.Target.from_depth_device(bufs[1].ptr, K, 0, ctx)
r = A.align_prepared(s, t, None, L.default_opts(max_iter=65))
nblk = (len(s) + 255) // 256
raw = np.zeros(nblk * 16, np.float64)
L.check(f(ctx.handle, raw.ctypes.data, len(raw)), "slab")
w = raw.view(np.int64).reshape(nblk * 4, 4)
t0, t1 = w[:, 0], w[:, 1]
# shader clocks from each wave's start (0: no such phase)
cert = w[:, 2] & 0xffffffff
entry = w[:, 2] >> 32
staged = w[:, 3] & 0xffffffff
scans = w[:, 3] >> 32
print(f"{nblk} workgroups, {len(w)} waves; {np.mean(entry > 0):.0%} enter the pixel search, "
      f"{np.mean(staged > 0):.0%} stage")
print(f"kernel span (first start -> last end): {(t1.max() - t0.min()) / 100:.1f} us")
print(f"wave start spread: {(t0.max() - t0.min()) / 100:.1f} us; end spread {(t1.max() - t1.min()) / 100:.1f} us")
lat = (t1 - t0) / 100
s = staged > 0
print("clocks from the wave's start, searching waves: to cert | reseed | window setup + first chunk trip | "
      "scans (+ further chunks) | latency us")
for q in (10, 50, 90, 99, 100):
    print(f"  p{q}: cert {np.percentile(cert[s], q):.0f}  reseed {np.percentile(entry[s] - cert[s], q):.0f}  "
          f"stage {np.percentile(staged[s] - entry[s], q):.0f}  scans {np.percentile(scans[s] - staged[s], q):.0f}  "
          f"latency {np.percentile(lat[s], q):.1f}")
ns = ~s
for q in (50, 90, 99):
    print(f"  non-staging waves p{q}: cert {np.percentile(cert[ns], q):.0f}  latency {np.percentile(lat[ns], q):.1f} us")
srt = np.argsort(t0)
print("starts by decile (us from first):", [round((np.percentile(t0, p) - t0.min()) / 100, 1) for p in range(0, 101, 10)])
print("ends by decile (us from first start):", [round((np.percentile(t1, p) - t0.min()) / 100, 1) for p in range(0, 101, 10)])
