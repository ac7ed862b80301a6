"""CPU model of the path-relative sequential-sum maps (seqsum design study).

For one float32 chain v (s_{k+1} = fl(s_k + v_k) from s_0 = +0, the
reference's `dst_mean += dst.GetPoint(j)`, align_icp.cpp:120) this checks,
block by block, the offset rule the GPU walker relies on:

  a block [p, q) run from a guessed start G + r*g0 (r < 2^M, g0 = the grid
  of G's binade) records its end E_r and the interval [LO_r, HI_r] of
  offsets d (multiples of a lattice L >= the grids it rounded on) for which
  every step of the run from G + r*g0 + d rounds exactly like the run from
  G + r*g0 (rounding steps: same binade; exact steps: still exact), so the
  true end is E_r + d.

and reports how often the true start falls outside the recorded interval
(the walker then adds that block serially), and whether E_r + d ever
differs from the true sequential sum (it must not).

    python tools/seqsum_sim.py [--iters 0,64]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def seq_prefix(v):
    acc = np.add.accumulate(v.astype(np.float32), dtype=np.float32)
    return np.concatenate([np.zeros(1, np.float32), acc])


def lsb32(r):
    """lowest set bit of float32 values as a float64 power of two (inf for 0)"""
    b = r.view(np.uint32).astype(np.int64)
    ex = (b >> 23) & 0xFF
    man = (b & 0x7FFFFF) | np.where(ex > 0, 0x800000, 0)
    tz = np.zeros_like(man)
    mm = man.copy()
    nz = mm != 0
    for _ in range(24):
        step = nz & ((mm & 1) == 0)
        tz += step
        mm = np.where(step, mm >> 1, mm)
    e = np.where(ex > 0, ex, 1) - 150 + tz
    return np.where(nz, np.ldexp(1.0, e.astype(np.int32)), np.inf)


def block_runs(v, starts, ends, S0, g0):
    """run every (block, residue) path; S0 [nb, R] float32 starts"""
    nb, R = S0.shape
    lens = ends - starts
    L = int(lens.max()) if nb else 0
    s = S0.copy()
    LO = np.full((nb, R), -np.inf)
    HI = np.full((nb, R), np.inf)
    need = np.zeros((nb, R))
    g0b = np.broadcast_to(g0[:, None], (nb, R))
    for k in range(L):
        act = (k < lens)[:, None]
        idx = np.minimum(starts + k, len(v) - 1)
        x = np.broadcast_to(v[idx][:, None], (nb, R)).astype(np.float32)
        r = (s + x).astype(np.float32)
        bb = (r - s).astype(np.float32)
        err = ((s - (r - bb)).astype(np.float32) + (x - bb).astype(np.float32)).astype(np.float32)
        exact = err == 0
        yd = r.astype(np.float64) + err.astype(np.float64)
        ay = np.abs(yd)
        _, fe = np.frexp(np.where(ay > 0, ay, 1.0))
        e = fe - 1
        lo_e = np.ldexp(1.0, e)
        hi_e = np.ldexp(1.0, e + 1)
        g = np.ldexp(1.0, e - 23)
        tie = np.abs(err.astype(np.float64)) == g / 2
        dlo_r = np.where(yd > 0, lo_e - yd, -hi_e - yd) + g
        dhi_r = np.where(yd > 0, hi_e - yd, -lo_e - yd) - g
        need_r = np.where(tie, 2 * g, g)
        q = np.minimum(lsb32(r), np.maximum(g0b, g))
        lim = q * 2.0 ** 24
        dlo_e = -lim - yd
        dhi_e = lim - yd
        lo = np.where(exact, dlo_e, dlo_r)
        hi = np.where(exact, dhi_e, dhi_r)
        LO = np.where(act, np.maximum(LO, lo), LO)
        HI = np.where(act, np.minimum(HI, hi), HI)
        need = np.where(act, np.maximum(need, np.where(exact, g, need_r)), need)
        s = np.where(act, r, s)
    return s, LO, HI, need


def guesses(v, A, starts, ends, G):
    """drift-corrected guesses: the chained float32 increments of unmonitored
    runs from the fp64 guesses"""
    s = G.copy()
    L = int((ends - starts).max())
    for k in range(L):
        act = k < ends - starts
        x = v[np.minimum(starts + k, len(v) - 1)]
        s = np.where(act, (s + x).astype(np.float32), s)
    inc = s.astype(np.float64) - G.astype(np.float64)
    return np.concatenate([[0.0], np.cumsum(inc)[:-1]])


def simulate(v, W=64, M=3, SW=64, verbose=True, refine=False, lattice="suffix"):
    v = v.astype(np.float32)
    n = len(v)
    T = seq_prefix(v)
    A = np.concatenate([[0.0], np.cumsum(v.astype(np.float64))])
    nw = (n + W - 1) // W
    p = np.zeros(nw + 1, np.int64)
    for w in range(1, nw):
        seg = np.abs(A[w * W:min((w + 1) * W, n)])
        p[w] = w * W + int(np.argmax(seg))
    p[nw] = n
    starts, ends = p[:-1], p[1:]
    G = A[starts].astype(np.float32)
    G[0] = 0.0
    if refine:
        G = guesses(v, A, starts, ends, G).astype(np.float32)
        G[0] = 0.0
    aG = np.abs(G.astype(np.float64))
    _, fe = np.frexp(np.where(aG > 0, aG, 1.0))
    g0 = np.where(aG > 0, np.ldexp(1.0, fe - 1 - 23), 2.0 ** -149)
    R = 1 << M
    # a guess just above a power of two: candidates from the top of the binade below
    top = np.ldexp(1.0, fe - 1 + 1)
    up = (np.abs(G.astype(np.float64)) >= top) & (aG > 0)
    G = np.where(up, np.sign(G) * (top - R * g0), G).astype(np.float32)
    S0 = (G.astype(np.float64)[:, None] + np.arange(R)[None, :] * g0[:, None]).astype(np.float32)
    assert np.all(S0.astype(np.float64) == G.astype(np.float64)[:, None] + np.arange(R)[None, :] * g0[:, None])
    E, LO, HI, need = block_runs(v, starts, ends, S0, g0)
    # lattice: suffix max of the needed lattice within each superwindow
    Lneed = np.maximum(need.max(1), g0)
    Lw = Lneed.copy()
    for w in range(nw - 2, -1, -1):
        if lattice == "suffix" and (w + 1) % SW != 0:
            Lw[w] = max(Lw[w], Lw[w + 1])
    m = np.round(np.log2(Lw / g0)).astype(int)
    # the true starts
    S = T[starts].astype(np.float64)
    d = S - G.astype(np.float64)
    k = d / g0
    ongrid = k == np.round(k)
    ki = np.round(k).astype(np.int64)
    bad_m = m > M
    mm = np.minimum(m, M)
    rr = ki & ((1 << mm) - 1)
    dp = (ki - rr) * g0
    Er = E[np.arange(nw), rr].astype(np.float64)
    ok = ongrid & ~bad_m & (LO[np.arange(nw), rr] <= dp) & (dp <= HI[np.arange(nw), rr])
    ok[0] = True  # exact start
    pred = Er + dp
    wrong = ok & (pred != T[ends].astype(np.float64))
    nfail = int((~ok).sum())
    if verbose == 2:
        for w in np.nonzero(~ok)[0][:40]:
            r = rr[w]
            print(f"   blk {w} start {S[w]:.6g} G {G[w]:.6g} d {d[w]:.3g} g0 {g0[w]:.3g} ongrid {ongrid[w]} "
                  f"m {m[w]} need/g0 {need[w].max()/g0[w]:.3g} win [{LO[w, r]:.3g},{HI[w, r]:.3g}] dp {dp[w]:.3g} "
                  f"len {ends[w]-starts[w]}")
    sw = np.arange(nw) // SW
    fails_sw = np.bincount(sw[~ok], minlength=sw.max() + 1)
    if verbose:
        print(f"  n={n} blocks={nw} fail={nfail} (off-grid {int((~ongrid).sum())}, m>{M} "
              f"{int(bad_m.sum())}, window {int((~ok & ongrid & ~bad_m).sum())}) WRONG={int(wrong.sum())}")
        print(f"  m histogram {np.bincount(m)[:8].tolist()}  superwindows {len(fails_sw)} with fails "
              f"{np.bincount(fails_sw).tolist()}")
        dd = np.abs(d)
        print(f"  |guess error| median {np.median(dd):.3g} max {dd.max():.3g};"
              f" window width median {np.median((HI - LO)[:, 0]):.3g}")
    return nfail, int(wrong.sum()), fails_sw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", default="0,8,64")
    ap.add_argument("--M", type=int, default=3)
    ap.add_argument("--W", type=int, default=64)
    ap.add_argument("--SW", type=int, default=64)
    ap.add_argument("--refine", action="store_true")
    ap.add_argument("--lattice", default="suffix")
    a = ap.parse_args()
    from oracle import oracle as O
    from realsensetracker_amd import driver
    K = driver.intrinsics(640, 480)
    da, db, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    pa, pb = O.unproject(da, K4), O.unproject(db, K4)
    tree = O.KDTree(pa)
    its = [int(x) for x in a.iters.split(",")]
    _, _, _, tr = O.align_icp(pb, pa, max(its) + 1, tree=tree, trace=True)
    for it in its:
        T = np.eye(4, dtype=np.float32) if it == 0 else tr["pose"][it - 1]
        q = (pb @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
        idx, d2 = tree.query(q)
        corr = pa[idx]
        print(f"iteration {it}")
        for c, name in enumerate("xyz"):
            print(f" chain {name}")
            simulate(corr[:, c], W=a.W, M=a.M, SW=a.SW, refine=a.refine, lattice=a.lattice)
        print(" chain cost")
        simulate(d2, W=a.W, M=a.M, SW=a.SW, refine=a.refine, lattice=a.lattice)


if __name__ == "__main__":
    main()
