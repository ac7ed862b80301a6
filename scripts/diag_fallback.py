"""Which fallback strategy disagrees with the oracle, and how."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
from oracle import oracle as O
from realsensetracker_amd import align as A, driver
from test_gpu_parity import _fallback

ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(3)
da, db, _ = driver.make_pair(sc, K, seed=31)
pa = driver.unproject(da, K, ctx=ctx); pb = driver.unproject(db, K, ctx=ctx)
t = A.Target.build(pa, ctx); tree = O.KDTree(pa)
rng = np.random.default_rng(2)
sel = rng.choice(len(pb), 3000, replace=False)
off = rng.normal(size=(3000, 3)).astype(np.float32)
off *= (10 ** rng.uniform(-3, np.log10(0.5), 3000)).astype(np.float32)[:, None] / np.linalg.norm(off, axis=1, keepdims=True)
q = (pb[sel] + off).astype(np.float32)
oi, od = tree.query(q)
gi0, _ = tree.query(pb[sel])
for mode in (0, 2, 3, 23, 100, 101, 102):
    for wn, warm in (("good", gi0.astype(np.int32)), ("rand", rng.integers(0, len(pa), 3000).astype(np.int32))):
        gi, gd, path = _fallback(ctx, t, q, warm, mode)
        bad = np.nonzero(gd != od)[0]
        print(f"mode {mode} warm {wn}: paths {np.bincount(path, minlength=4).tolist()} bad {len(bad)}"
              f" bad-paths {np.bincount(path[bad], minlength=4).tolist() if len(bad) else []}")
        for b in bad[:3]:
            print("   ", b, "od", od[b], "gd", gd[b], "oi", oi[b], "gi", gi[b], "|off|", np.linalg.norm(off[b]))
gi, gd = t.query(q)
print("k_query_nn (per-lane descend) bad:", int(np.sum(gd != od)))
gi, gd = t.query_warm(q, gi0.astype(np.int32))
print("k_query_nn_warm (nn_wave_region) bad:", int(np.sum(gd != od)))
gi, gd, path = _fallback(ctx, t, q, None, 0)
print("walk from root bad:", int(np.sum(gd != od)))
