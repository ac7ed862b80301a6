"""Does RST_SUM_FP64 (fp64 partial sums) meet the north_star's 1e-4 gate
against the reference's arithmetic (its fp32 sequential sums)?  Writes
tests/golden/fp64_gate.json (committed; read by tests/test_fp64_gate.py).

For each pair: the oracle's AlignIcp3d restatement (oracle/rst_oracle.c,
align_icp.cpp:73-161) twice -- sum_mode 0, the reference's fp32 sequential
dst_mean / cost / centroid sums (:85-86,113,120-122), and sum_mode 1, fp64
sums (the device's RST_SUM_FP64 arithmetic) -- and the pose error between
them (rad, m).  Pairs: bench.py's own workloads --
  * configs[1]: 64 consecutive pairs (k, k - 1) of the 640x480 stream
    (render_frames(seed=0): trajectory(k), noise seed k);
  * configs[2]: the 1280x720 stream's first pair;
  * configs[3]: the 1000x1000 sharded pair (frames 1 -> 0).
128 iterations each (rs_replay_app.cpp:246-251).  About 5 minutes on 8
threads (the oracle's NN loop is OpenMP; the sums stay sequential).

    python tests/golden/make_fp64_gate.py [--pairs 64]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from oracle import oracle as O  # noqa: E402
from posemetric import pose_err  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

OUT = Path(__file__).resolve().parent / "fp64_gate.json"


def frames(w, h, n):
    """bench.py render_frames(seed=0, n, K, stride=1)."""
    K = driver.intrinsics(w, h)
    sc = driver.SyntheticScene(0)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    return [O.unproject(sc.render(sc.trajectory(i), K, noise_seed=i), K4) for i in range(n)]


def gate_case(src, dst, iters=128):
    tree = O.KDTree(dst)
    ok0, T0, c0, _ = O.align_icp(src, dst, iters, tree=tree, sum_mode=0)
    ok1, T1, c1, _ = O.align_icp(src, dst, iters, tree=tree, sum_mode=1)
    e = pose_err(T0, T1)
    return {"n": len(src), "m": len(dst), "rad": e[0], "m_err": e[1], "ok_ref": ok0, "ok_fp64": ok1,
            "cost_ref": c0, "cost_fp64": c1,
            "pose_ref": T0.tolist(), "pose_fp64": T1.tolist()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    O.set_threads(a.threads)
    t0 = time.time()
    out = {"iters": 128, "stream_640x480": [], "gate": 1e-4}
    f = frames(640, 480, a.pairs + 1)
    for k in range(1, a.pairs + 1):
        c = gate_case(f[k], f[k - 1])
        c["pair"] = k
        out["stream_640x480"].append(c)
        print(f"640x480 pair {k}: {c['rad']:.3g} rad {c['m_err']:.3g} m ({time.time() - t0:.0f} s)",
              flush=True)
    f = frames(1280, 720, 2)
    out["stream_1280x720"] = gate_case(f[1], f[0])
    print("1280x720:", out["stream_1280x720"]["rad"], out["stream_1280x720"]["m_err"], flush=True)
    f = frames(1000, 1000, 2)
    out["sharded_1000x1000"] = gate_case(f[1], f[0])
    print("1000x1000:", out["sharded_1000x1000"]["rad"], out["sharded_1000x1000"]["m_err"], flush=True)
    allc = out["stream_640x480"] + [out["stream_1280x720"], out["sharded_1000x1000"]]
    out["max_rad"] = max(c["rad"] for c in allc)
    out["max_m"] = max(c["m_err"] for c in allc)
    out["all_within_gate"] = bool(out["max_rad"] <= 1e-4 and out["max_m"] <= 1e-4 and
                                  all(c["ok_ref"] == c["ok_fp64"] for c in allc))
    out["seconds"] = time.time() - t0
    OUT.write_text(json.dumps(out, indent=1) + "\n")
    print(f"max {out['max_rad']:.3g} rad {out['max_m']:.3g} m, within gate: {out['all_within_gate']}")


if __name__ == "__main__":
    main()
