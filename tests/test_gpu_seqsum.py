"""RST_SUM_REF's sequential float32 sums (align_icp.cpp:113,120-122;
point_cloud_utils.cpp:94-96) -- the parallel exact kernels of seqsum.hip
against numpy's sequential float32 accumulate (np.add.accumulate with a
float32 dtype adds left to right, one rounding per element: the
reference's `+=` loop), bit for bit, and against the one-wavefront serial
chain (k_seq_sum4) they replace."""
import ctypes as C

import numpy as np
import pytest

from realsensetracker_amd import _lib as L
from realsensetracker_amd import align as A
from realsensetracker_amd import driver
from seqsum_cases import cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return A.get_context(0)


def _fn():
    f = L.lib().rst_debug_seq_sum
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, L.c_float_p, C.c_int64, C.c_int, C.c_int, L.c_float_p,
                  C.POINTER(C.c_float), C.c_void_p]
    return f


def seq_sum(ctx, x, serial=0, reps=1, stats=None):
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros(4, np.float32)
    ms = C.c_float(0)
    sp = stats.ctypes.data if stats is not None else None
    L.check(_fn()(ctx.handle, L.fptr(x), len(x), serial, reps, L.fptr(out), C.byref(ms), sp),
            "seq_sum")
    return out, ms.value


def want(x):
    # from a +0 start (the reference's Zero() vector): +0 + -0 = +0
    x = np.concatenate([np.zeros((1, 4), np.float32), np.asarray(x, np.float32)])
    return np.add.accumulate(x, axis=0, dtype=np.float32)[-1]


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return np.array_equal(a.view(np.uint32), b.view(np.uint32)) or \
        np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
            np.where(np.isnan(a), 0, a).view(np.uint32), np.where(np.isnan(b), 0, b).view(np.uint32))


CASES = cases()


PATHS = {"auto": 0, "maps": 2, "replay": 3, "small": 4}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("name", sorted(CASES))
def test_parallel_seq_sum_bitexact(ctx, name, path):
    """Every edge case by every path (the map pipeline and the one-wavefront
    replay k_sq_serial, forced at any size; the one-workgroup-per-chain
    k_sq_small, forced up to its 16384 elements) and by the size rule."""
    x = CASES[name]
    got, _ = seq_sum(ctx, x, serial=PATHS[path])
    assert same(got, want(x)), (name, path, got, want(x))


@pytest.mark.parametrize("n", [1, 31, 1023, 1024, 1025, 2047, 2048, 2049, 15_237, 40_000])
def test_replay_tile_edges(ctx, n):
    """k_sq_serial around its 1024-element tiles and 32-element groups (the
    padded tail), with large-magnitude, cancelling and non-finite-free
    chains: bit-exact against numpy's sequential float32 sums, and equal to
    the map pipeline's."""
    rng = np.random.default_rng(n)
    x = (rng.standard_normal((n, 4)) * np.array([1e3, 1e-3, 1.0, 1e6])).astype(np.float32)
    x[:, 2] -= np.float32(0.25)
    a, _ = seq_sum(ctx, x, serial=3)
    b, _ = seq_sum(ctx, x, serial=2)
    assert same(a, want(x)) and same(b, want(x)), (n, a, b, want(x))


def test_parallel_seq_sum_frames(ctx):
    """Real 640x480 clouds in pixel order (the order the reference sums:
    the source in its original order, dst[nbr_i] for i ascending), both
    frames of a pair and their squared ranges as a cost-like chain."""
    K = driver.intrinsics(640, 480)
    for seed in (10, 11):
        da, db, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=seed)
        for d in (da, db):
            p = driver.unproject(d, K)
            x = np.concatenate([p, (p * p).sum(1, keepdims=True)], 1).astype(np.float32)
            got, _ = seq_sum(ctx, x)
            assert same(got, want(x)), (got, want(x))
            # shifted so that the x chain starts far from zero, then crosses it
            y = x.copy()
            y[:, 0] -= np.float32(np.mean(x[:, 0]))
            got, _ = seq_sum(ctx, y)
            assert same(got, want(y))


def test_parallel_matches_serial_kernel_and_is_faster(ctx):
    K = driver.intrinsics(640, 480)
    da, _, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
    p = driver.unproject(da, K)
    x = np.concatenate([p, (p * p).sum(1, keepdims=True)], 1).astype(np.float32)
    a, ms_par = seq_sum(ctx, x, serial=0, reps=20)
    b, ms_ser = seq_sum(ctx, x, serial=1, reps=3)
    c, ms_rep = seq_sum(ctx, x, serial=3, reps=3)
    assert same(a, b) and same(a, c)
    print(f"\nseq sums of {len(x)} float4: parallel {ms_par * 1e3:.1f} us, "
          f"serial {ms_ser * 1e3:.1f} us, replay {ms_rep * 1e3:.1f} us")
    assert ms_par < ms_ser and ms_par < ms_rep


def test_replay_chosen_where_faster(ctx):
    """The size rule: at 4096 elements (below RST_SQ_SERIAL_MAX's 8192) the
    replay, the product's choice there, is faster than the map pipeline
    (measured 23 vs 50 us, r05a); at 640x480 sizes the map pipeline is (the
    test above)."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((4096, 4)).astype(np.float32)
    a, ms_auto = seq_sum(ctx, x, serial=0, reps=20)
    b, ms_maps = seq_sum(ctx, x, serial=2, reps=20)
    c, ms_rep = seq_sum(ctx, x, serial=3, reps=20)
    assert same(a, want(x)) and same(b, a) and same(c, a)
    print(f"\nseq sums of 4096 float4: auto {ms_auto * 1e3:.1f} us, maps {ms_maps * 1e3:.1f} us, "
          f"replay {ms_rep * 1e3:.1f} us")
    assert ms_rep < ms_maps


@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 255, 256, 257, 1023, 4097, 8191, 15_239, 16_383, 16_384])
@pytest.mark.parametrize("kind", ["normal", "drift", "ties"])
def test_small_kernel_edges(ctx, n, kind):
    """k_sq_small (one workgroup per chain: leaf maps in LDS, 16-block
    group maps, one walking wavefront) around its window, group and size
    edges, on chains whose sums grow through many binades (the z-like
    drift), cross zero, and tie on every step: bit-exact against numpy's
    sequential float32 sums and equal to the map pipeline's."""
    rng = np.random.default_rng(1000 + n)
    if kind == "normal":
        x = (rng.standard_normal((n, 4)) * np.array([1e3, 1e-3, 1.0, 1e6])).astype(np.float32)
        x[:, 2] -= np.float32(0.25)
    elif kind == "drift":  # coordinates of a 0.3-5 m scene: sums up to ~8e4, crossing binades
        x = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(0.3, 5.0, n),
                      rng.uniform(0, 1e-4, n)], 1).astype(np.float32)
    else:  # a half-ulp tie at every step of the first chain
        x = np.zeros((n, 4), np.float32)
        x[:, 0] = np.float32(1.0)
        x[1:, 0] = np.float32(2.0 ** -24)
        x[:, 1] = np.float32(3.0)
        x[:, 2] = rng.choice(np.array([0.5, -0.25, 2.0 ** -30], np.float32), n)
        x[:, 3] = np.float32(0.1)
    a, _ = seq_sum(ctx, x, serial=4)
    b, _ = seq_sum(ctx, x, serial=2)
    assert same(a, want(x)) and same(b, want(x)), (n, kind, a, b, want(x))


def test_small_kernel_timing(ctx):
    """The size rule between the replay, k_sq_small and the map pipeline at
    the reference callers' sizes (rs_replay_app.cpp:246-251: ~15k points at
    5 cm; ~4k at the tracker's 10 cm): k_sq_small is faster than the map
    pipeline at 15k."""
    rng = np.random.default_rng(6)
    res = {}
    for n in (1024, 2048, 4096, 8192, 15_239):
        x = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(0.3, 5.0, n),
                      rng.uniform(0, 1e-4, n)], 1).astype(np.float32)
        t = {}
        for name, code in (("small", 4), ("maps", 2), ("replay", 3), ("auto", 0)):
            got, ms = seq_sum(ctx, x, serial=code, reps=20)
            assert same(got, want(x)), (n, name)
            t[name] = ms * 1e3
        res[n] = t
        print(f"\nseq sums of {n} float4: " + ", ".join(f"{k} {v:.1f} us" for k, v in t.items()))
    assert res[15_239]["small"] < res[15_239]["maps"]


def test_wave_scan_dpp(ctx):
    """The DPP scans behind the maps' guesses (seqsum.hip wave_scan_incl,
    block_scan_excl: row_shr / row_bcast lane moves, no LDS): an inclusive
    and an exclusive scan of one wave of doubles and the total, against
    numpy's -- their fp64 rounding differs from a serial sum (guesses only:
    the sums themselves stay exact whatever the prefixes), so to 1e-12."""
    import ctypes as C
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.normal(size=64) * 1e3, rng.uniform(-2, 3, 64)]).astype(np.float64)
    out = np.zeros(129, np.float64)
    f = L.lib().rst_debug_wave_scan
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]
    L.check(f(ctx.handle, x.ctypes.data, out.ctypes.data), "rst_debug_wave_scan")
    inc = np.cumsum(x[:64])
    exc = np.concatenate([[0.0], np.cumsum(x[64:])[:-1]])
    tol = 1e-12 * np.abs(x).sum()
    assert np.max(np.abs(out[:64] - inc)) <= tol, out[:64] - inc
    assert np.max(np.abs(out[64:128] - exc)) <= tol, out[64:128] - exc
    assert abs(out[128] - x[64:].sum()) <= tol
