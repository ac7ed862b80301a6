"""Where the one-wavefront replay (k_sq_serial) beats the map pipeline:
device time per sequential-sum launch of n float4 by both paths
(rst_debug_seq_sum serial = 2 / 3), with the sums checked equal.  Sets
RST_SQ_SERIAL_MAX's default (seqsum.hip kSerDefault).
  python tools/seq_serial_sweep.py"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from realsensetracker_amd import align as A  # noqa: E402
from test_gpu_seqsum import same, seq_sum  # noqa: E402

ctx = A.get_context(0)
rng = np.random.default_rng(1)
print(f"{'n':>8} {'maps_us':>9} {'replay_us':>10} {'ns/elem':>8}")
for n in (2048, 4096, 8192, 15_000, 24_576, 32_768, 49_152, 65_536, 98_304, 300_000):
    x = (rng.standard_normal((n, 4)) + 2.0).astype(np.float32)
    a, tm = seq_sum(ctx, x, serial=2, reps=30)
    b, tr = seq_sum(ctx, x, serial=3, reps=30)
    assert same(a, b), n
    print(f"{n:8d} {tm * 1e3:9.1f} {tr * 1e3:10.1f} {tr * 1e6 / n:8.2f}", flush=True)
