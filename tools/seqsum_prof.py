"""Time the RST_SUM_REF sequential sums (seqsum.hip) on a 640x480 frame:
parallel path vs the serial chain; run under rocprofv3 --kernel-trace
--stats for the per-kernel split."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import numpy as np  # noqa: E402

from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402
from test_gpu_seqsum import seq_sum, want, same  # noqa: E402

ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
da, _, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
p = driver.unproject(da, K)
x = np.concatenate([p, (p * p).sum(1, keepdims=True)], 1).astype(np.float32)
for serial, reps in ((0, 20), (1, 2)):
    out, ms = seq_sum(ctx, x, serial=serial, reps=reps)
    print("serial" if serial else "parallel", f"{ms * 1e3:.1f} us", same(out, want(x)))
st = np.zeros((8, 8), np.int32)
seq_sum(ctx, x, stats=st)
print("walk stats per chain [superblock tries, hits, group tries, hits, leaf tries, hits, serial blocks, walker clocks]")
print(st[:4])
print('bound-check error bits', st[4, 0], 'walker clocks waiting for map chunks', st[4, 1:5].tolist())
print('walker clocks at the start of chunks 0-3 per chain', st[5:7].reshape(4, 4).tolist())
print('chain 0 first descent phases (clocks from its start: groups loaded, group walk, leaves loaded, leaf walk, serial block, end)', st[7, 1:7].tolist())
for c in range(4):
    y = np.zeros_like(x)
    y[:, c] = x[:, c]
    out, ms = seq_sum(ctx, y, serial=0, reps=10)
    print("chain", c, f"{ms * 1e3:.1f} us", same(out, want(y)))
