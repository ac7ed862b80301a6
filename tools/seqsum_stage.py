"""Debug the sequential-sum kernels one at a time (rst_debug_seq_stages):
run the front kernel alone (or up to the maps / the walk), synchronised
after each, and compare its tables with the host emulation
(tests/cpp/seqsum_emu.cpp, built here by tests/seqsum_emu.py).

    python tools/seqsum_stage.py [stages] [case]     (stages: 1 front, 3, 7)
"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402

KW, KGW, KKW = 16, 16, 16


def layout(n, nch=4):
    nb = (n + KW - 1) // KW
    ng = (nb + KGW - 1) // KGW
    nk = (ng + KKW - 1) // KKW
    ns = (n + 63) & ~63
    off = 0
    out = {}
    for name, size in (("ttot2", 8 * 2 * 4 * 4 * nk), ("soa", 4 * nch * ns), ("wflg", nch * nb),
                       ("err", 4), ("ttot", 8 * nch * 4 * nk), ("bs", 4 * nch * (nb + 1)), ("gs", 4 * nch * (ng + 1)),
                       ("ks", 4 * nch * (nk + 1)), ("inc", 8 * nch * nb), ("ipre", 8 * nch * nb), ("tinc", 8 * nch * nk),
                       ("leaf", 64 * nch * nb), ("grp", 256 * nch * ng), ("sbm", 1024 * nch * nk), ("clk", 64 * nch * nk)):
        out[name] = off
        off += (size + 255) & ~255
    return out, nb, ng, nk, off


def run(x, stages, nch=4):
    lib = L.lib()
    f = lib.rst_debug_seq_stages
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, L.c_float_p, C.c_int64, C.c_int, C.c_int, L.c_float_p, C.c_void_p,
                  C.c_int64, C.POINTER(C.c_int)]
    g = lib.rst_debug_seq_ws_bytes
    g.restype = C.c_int64
    g.argtypes = [C.c_int64]
    ctx = A.get_context(0)
    n = len(x)
    wsb = g(n)
    ws = np.zeros(wsb, np.uint8)
    out = np.zeros(4, np.float32)
    failed = C.c_int(0)
    st = f(ctx.handle, L.fptr(np.ascontiguousarray(x, np.float32)), n, nch, stages, L.fptr(out),
           ws.ctypes.data, wsb, C.byref(failed))
    return st, failed.value, out, ws


def main():
    stages = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    case = sys.argv[2] if len(sys.argv) > 2 else "alternating"
    if case == "frame":
        from realsensetracker_amd import driver
        K = driver.intrinsics(640, 480)
        da, _, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
        p = driver.unproject(da, K)
        x = np.concatenate([p, (p * p).sum(1, keepdims=True)], 1).astype(np.float32)
    else:
        from seqsum_cases import cases
        x = cases()[case]
    st, failed, out, ws = run(x, stages)
    print(f"case {case} n={len(x)} stages {stages}: status {st}, failed stage {failed}, out {out}")
    off, nb, ng, nk, total = layout(len(x))
    err = ws[off["err"]:off["err"] + 4].view(np.int32)[0]
    print("err bits", err)
    clk = ws[off["clk"]:off["clk"] + 64 * 4 * nk].view(np.int64).reshape(4, nk, 8)
    if stages & 2:
        t = clk.astype(np.float64)
        # k_sq_build's stamps (the single-stream maps: leaf runs, then
        # wavefront 0's composites): start 0, staged 1, leaves done 6;
        # composites start 2, group composites done 3, group maps stored 4,
        # superblock 5 (the batched k_sq_leaves_b / k_sq_comp_b stamp alike)
        d = np.stack([t[..., 1] - t[..., 0], t[..., 6] - t[..., 1], t[..., 2] - t[..., 6],
                      t[..., 3] - t[..., 2], t[..., 4] - t[..., 3], t[..., 5] - t[..., 4]], axis=2)
        names = ["staging", "leaves (+ extra candidates)", "barrier", "group lattice + composites",
                 "group store", "superblock"]
        print("map kernel phases (clocks, mean / max over superblocks):",
              {nm: (round(d[:, :, i].mean()), int(d[:, :, i].max())) for i, nm in enumerate(names)})
    from seqsum_emu import emulate_tables
    for c in range(4):
        bs = ws[off["bs"]:].view(np.int32)[c * (nb + 1):(c + 1) * (nb + 1)]
        gs = ws[off["gs"]:].view(np.int32)[c * (ng + 1):(c + 1) * (ng + 1)]
        ks = ws[off["ks"]:].view(np.int32)[c * (nk + 1):(c + 1) * (nk + 1)]
        inc = ws[off["inc"]:].view(np.float64)[c * nb:(c + 1) * nb]
        ebs, egs, eks, einc = emulate_tables(x, c)
        print(f" chain {c}: bs {np.array_equal(bs, ebs)} gs {np.array_equal(gs, egs)} ks {np.array_equal(ks, eks)}"
              f" inc max|d| {np.max(np.abs(inc - einc)):.3g}  ks {ks[:6]}... vs {eks[:6]}")
        if not np.array_equal(ks, eks):
            bad = np.nonzero(ks != eks)[0]
            print("   ks differs at", bad[:10], ks[bad[:10]], eks[bad[:10]])


if __name__ == "__main__":
    main()
