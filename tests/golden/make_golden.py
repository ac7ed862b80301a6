"""Generate tests/golden/*.npz (run in the build container; committed).

The reference ships no tests or fixtures and cannot be built
here, so the golden vectors come from the C oracle
(oracle/rst_oracle.c) and are only written after the independent numpy/scipy
restatement (tests/np_restate.py) reproduces them:
  * NN indices / squared distances of iteration 0: identical;
  * fp64 covariances of iterations 0 and 1: identical to 1e-9 relative;
  * poses after 1, 8 and 128 iterations: within 2e-6.
Inputs are seeded synthetic frame pairs from the product's own scene
renderer (host code, librst_align.so) and RandomSource-style clouds.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from oracle import oracle as O  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402
import np_restate as NPR  # noqa: E402
from posemetric import pose_err  # noqa: E402

OUT = Path(__file__).resolve().parent


def icp_case(name, src, dst, T_gt, max_iter=128):
    ok, T, mc, tr = O.align_icp(src, dst, max_iter, trace=True)
    ok64, T64, mc64, _ = O.align_icp(src, dst, max_iter, sum_mode=1)
    okn, Tn, mcn, trn = NPR.align_icp(src, dst, max_iter, trace=True)
    assert np.array_equal(tr["nn_idx0"], trn["nn_idx0"]), name
    assert np.array_equal(tr["nn_d20"], trn["nn_d20"]), name
    for k in (0, 1):
        c, cn = tr["cov"][k], trn["cov"][k]
        assert np.allclose(c, cn, rtol=1e-9, atol=1e-12), (name, k, c, cn)
    for k in (0, 7, max_iter - 1):
        e = pose_err(tr["pose"][k], trn["pose"][k])
        assert max(e) <= 2e-6, (name, k, e)
    assert ok == okn and abs(mc - mcn) <= 1e-6 * max(1.0, mc), (name, mc, mcn)
    print(f"{name}: n={len(src)} m={len(dst)} oracle==numpy ok; "
          f"fp32seq-vs-fp64 {pose_err(T, T64)}; vs gt {pose_err(T, T_gt)}")
    return {
        "src": src, "dst": dst, "T_gt": np.asarray(T_gt, np.float32),
        "nn_idx0": tr["nn_idx0"], "nn_d20": tr["nn_d20"],
        "cov0": tr["cov"][0], "cov1": tr["cov"][1], "dmean0": tr["dmean"][0],
        "cost": tr["cost"], "mu": tr["mu"],
        "pose1": tr["pose"][0], "pose8": tr["pose"][7], "pose_final": T,
        "mean_cost": np.float32(mc), "ok": np.bool_(ok),
        "pose_final_fp64": T64, "max_iter": np.int32(max_iter),
    }


def main():
    cases = {}
    # synthetic RGB-D pairs at reduced resolution (the oracle runs them in seconds)
    for (w, h, seed) in [(80, 60, 0), (120, 90, 1), (160, 120, 2)]:
        K = driver.intrinsics(w, h)
        sc = driver.SyntheticScene(seed)
        da, db, D = driver.make_pair(sc, K, seed=seed + 10)
        K4 = [K.fx, K.fy, K.cx, K.cy]
        pa, pb = O.unproject(da, K4), O.unproject(db, K4)
        name = f"pair_{w}x{h}_s{seed}"
        c = icp_case(name, pb, pa, D)
        # P2PLANE (build's own mode) on the same pair, with kNN-16 normals
        tree = O.KDTree(pa)
        na = O.compute_normals(pa, 16, tree=tree)
        it, T2, mc2 = O.align_p2plane(pb, pa, na, 30, 1e-6, 4e-4, 0.0, tree=tree)
        c.update({"normals_dst": na, "p2plane_pose": T2, "p2plane_iters": np.int32(it),
                  "p2plane_cost": np.float32(mc2), "depth_a": da, "depth_b": db,
                  "K4": np.asarray(K4, np.float32)})
        cases[name] = c
    # RandomSource-shaped cloud (data_source.hpp:22-41): uniform [-1,1]^3,
    # 128 and 2048 points, target = known rigid motion of the source
    rng = np.random.default_rng(7)
    for n in (128, 2048):
        src = rng.uniform(-1, 1, size=(n, 3)).astype(np.float32)
        D = driver.random_offset(rng, deg=(2, 5), cm=(2, 5))
        dst = (src.astype(np.float64) @ D[:3, :3].T + D[:3, 3]).astype(np.float32)
        cases[f"random_{n}"] = icp_case(f"random_{n}", src, dst, D)
    for name, c in cases.items():
        np.savez_compressed(OUT / f"{name}.npz", **c)
    print("wrote", len(cases), "fixtures to", OUT)


if __name__ == "__main__":
    main()
