"""GPU: the BASELINE configs at full size, against the oracle (test
infrastructure) -- the in-loop exactness of the reference-rounding mode at
640x480 (every iteration's sequential sums bit for bit), RST_SUM_REF at
1280x720, point-to-plane at 1280x720 (configs[2]) and the 3-level 1280x720
pyramid under hipGraph replay (configs[4]).

The loop under test is the reference's `AlignIcp3d`
(rs_tracker/align/src/align_icp.cpp:73-161) as the replay app calls it per
frame pair (rs_tracker/app/src/rs_replay_app.cpp:246-251)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O
from posemetric import pose_err
from realsensetracker_amd import _lib as L
from realsensetracker_amd import align as A
from realsensetracker_amd import driver

pytestmark = pytest.mark.gpu

THREADS = 16  # the oracle's OpenMP NN loop (same result at any thread count)


@pytest.fixture(scope="module")
def ctx():
    c = A.get_context(0)
    O.set_threads(THREADS)
    yield c
    O.set_threads(1)


def _frames(ctx, w, h, scene, seed, nlev=1, normals_k=0):
    """A depth pair of the synthetic stream, its device targets (levels
    0..nlev-1 prepared from the depth on the GPU) and the oracle's clouds of
    the same levels (every 2^l-th pixel of every 2^l-th row)."""
    K = driver.intrinsics(w, h)
    da, db, D = driver.make_pair(driver.SyntheticScene(scene), K, seed=seed)
    ba, bb = A.DeviceBuffer.from_array(da, ctx), A.DeviceBuffer.from_array(db, ctx)
    tl = A.Target.pyramid_from_depth_device(ba.ptr, K, nlev, normals_k, ctx)
    sl = A.Target.pyramid_from_depth_device(bb.ptr, K, nlev, 0, ctx)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    pa = [O.unproject(da, K4, stride=1 << lv) for lv in range(nlev)]
    pb = [O.unproject(db, K4, stride=1 << lv) for lv in range(nlev)]
    for lv in range(nlev):
        assert len(tl[lv]) == len(pa[lv]) and len(sl[lv]) == len(pb[lv])
    return sl, tl, pb, pa, D, (ba, bb)


def _seq_trace(ctx, n):
    out = np.zeros((n, 4), np.float32)
    f = L.lib().rst_debug_seq_trace
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_void_p, C.c_int32]
    L.check(f(ctx.handle, out.ctypes.data, n), "rst_debug_seq_trace")
    return out


def _enable_seq_trace(ctx, on):
    f = L.lib().rst_debug_enable_seq_trace
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_int]
    L.check(f(ctx.handle, int(on)), "rst_debug_enable_seq_trace")


def test_ref_inloop_sums_bitexact_640(ctx):
    """640x480 frame pair, frame targets (pixel windows + certificates +
    BVH fallback decide every iteration's correspondences), 128 iterations
    of RST_SUM_REF: in EVERY iteration the device's sequential sums of the
    correspondences' coordinates and of their d2 -- each one a function of
    all ~300k (index, d2) pairs of that iteration -- equal the reference
    arithmetic's bit for bit (dst_mean :113,122 and cost :120), so the
    loop's correspondences are the reference's in every iteration, not
    only its final pose."""
    sl, tl, pb, pa, _, keep = _frames(ctx, 640, 480, 5, 17)
    n = len(pb[0])
    _enable_seq_trace(ctx, True)
    try:
        r = A.align_prepared(sl[0], tl[0], None, L.default_opts(max_iter=128))
        tr = _seq_trace(ctx, 128)
    finally:
        _enable_seq_trace(ctx, False)
    assert r.ok and r.iterations == 128
    ok, To, mco, otr = O.align_icp(pb[0], pa[0], 128, tree=O.KDTree(pa[0]), trace=True, sum_mode=0)
    dmean = (tr[:, :3] / np.float32(n)).astype(np.float32)  # dst_mean /= n (:122)
    bad_d = np.flatnonzero(np.any(dmean.view(np.uint32) != otr["dmean"].view(np.uint32), axis=1))
    bad_c = np.flatnonzero(tr[:, 3].view(np.uint32) != otr["cost"].view(np.uint32))
    assert bad_d.size == 0, f"dst_mean differs from iteration {bad_d[:5]}"
    assert bad_c.size == 0, f"cost differs from iteration {bad_c[:5]}"
    e = pose_err(r.pose, To)
    print(f"640x480 in-loop trace: 128/128 iterations bit-exact; pose vs oracle {e}")
    assert max(e) <= 1e-6, e  # the north_star gate is 1e-4; measured 0 (r03e)
    assert abs(r.mean_cost - mco) <= 1e-6 * max(1.0, abs(mco))


def test_ref_720p_matches_reference_arithmetic(ctx):
    """BASELINE configs[2] size (1280x720, ~900k points) in the drop-in
    default mode: 128 iterations within the north_star's 1e-4 of the
    reference arithmetic (the oracle with its fp32 sequential sums)."""
    sl, tl, pb, pa, _, keep = _frames(ctx, 1280, 720, 3, 11)
    assert len(pb[0]) > 800_000
    r = A.align_prepared(sl[0], tl[0], None, L.default_opts(max_iter=128))
    ok, To, mco, _ = O.align_icp(pb[0], pa[0], 128, tree=O.KDTree(pa[0]), sum_mode=0)
    e = pose_err(r.pose, To)
    print(f"1280x720 RST_SUM_REF vs reference arithmetic: {e}, cost {r.mean_cost} vs {mco}")
    assert r.ok == ok
    assert max(e) <= 1e-6, e  # the north_star gate is 1e-4; measured 0 (r03e)
    assert abs(r.mean_cost - mco) <= 1e-6 * max(1.0, abs(mco))


@pytest.mark.parametrize("normals_k", [-2, 16])
def test_p2plane_720p(ctx, normals_k):
    """configs[2]: point-to-plane at 1280x720 from frame targets (image-grid
    or kNN-16 normals): the device loop equals its C restatement run with
    the device's normals, and recovers the frames' known motion."""
    sl, tl, pb, pa, D, keep = _frames(ctx, 1280, 720, 7, 33, normals_k=normals_k)
    o = L.default_opts(mode=L.RST_P2PLANE, max_iter=30)
    r = A.align_prepared(sl[0], tl[0], None, o)
    assert r.ok
    nrm = tl[0].normals()  # in the oracle cloud's order (original order)
    it, To, _ = O.align_p2plane(pb[0], pa[0], nrm, max_iter=30, eps=o.p2plane_eps,
                                mu=o.p2plane_mu, max_dist=o.p2plane_max_dist,
                                tree=O.KDTree(pa[0]))
    e = pose_err(r.pose, To)
    g = pose_err(r.pose, D)
    print(f"P2PLANE 1280x720 normals_k={normals_k}: {r.iterations} vs {it} iterations, "
          f"vs restatement {e}, vs truth {g}")
    assert max(e) <= 1e-6, e  # measured 0 (r03e): the same fp64 system, solve and steps
    assert g[0] < 1e-4 and g[1] < 3.5e-4, g  # measured 3-4e-5 rad, 2.0-2.5e-4 m (r03e)


@pytest.mark.parametrize("sum_mode", [L.RST_SUM_REF, L.RST_SUM_FP64])
def test_pyramid_720p_graphs(ctx, sum_mode):
    """configs[4]: the 3-level 1280x720 pyramid (32 / 32 / 64 iterations,
    finest first -- the bench's) replayed as hipGraphs equals the oracle's
    level-by-level chain: within 1e-4 of the reference arithmetic in the
    drop-in mode, 2e-5 of the fp64-sum restatement in the fp64 mode; and the
    graph replay equals the stream launch bit for bit."""
    sl, tl, pb, pa, _, keep = _frames(ctx, 1280, 720, 2, 21, nlev=3)
    iters = [32, 32, 64]
    o = L.default_opts(sum_mode=sum_mode)
    gctx = A.Context(0)
    try:
        gctx.enable_graphs(True)
        gsl, gtl, _, _, _, gkeep = _frames(gctx, 1280, 720, 2, 21, nlev=3)
        r = A.align_pyramid(gsl, gtl, iters, None, o)
        r2 = A.align_pyramid(gsl, gtl, iters, None, o)  # the executables updated in place
    finally:
        gctx.close()
    rs = A.align_pyramid(sl, tl, iters, None, o)
    assert np.array_equal(r.pose, rs.pose) and np.array_equal(r2.pose, rs.pose)
    ok, To, _ = O.align_icp_pyramid(pb, pa, iters, sum_mode=0 if sum_mode == L.RST_SUM_REF else 1)
    e = pose_err(r.pose, To)
    print(f"1280x720 pyramid (graphs, sum_mode {sum_mode}) vs oracle chain: {e}")
    assert ok == r.ok
    assert max(e) <= 1e-6, e  # gates 1e-4 / 2e-5 by contract; measured 0 (r03e)


@pytest.mark.parametrize("voxel", [0.05, 0.1])
def test_callers_workload_ref_inloop(ctx, voxel):
    """The reference callers' own sizes (rs_replay_app.cpp:229,246-251:
    RemoveNans, DownsampleVoxel 0.05 of both clouds, the 4-argument
    AlignIcp3d 128): ~15k points, each chain's sums in one workgroup of
    k_sq_small (seqsum.hip: chains of <= 16,384 elements, maps and walk in
    LDS) -- every iteration's sums bit-exact again; at 10 cm (~4k points, the
    tracker's voxel, rs_tracker.cpp) the one-wavefront replay k_sq_serial
    takes the sums instead, bit-exact the same way."""
    K = driver.intrinsics(640, 480)
    da, db, _ = driver.make_pair(driver.SyntheticScene(0), K, seed=10)
    # the recorded clouds keep every pixel, invalid ones at the origin
    # (data_source_rs.cpp:89-90 writes 0 for NaN); a few NaNs as well
    raw = [driver.unproject(d, K, keep_invalid=True) for d in (da, db)]
    for r in raw:
        r[::997] = np.nan
    cur = A.DownsampleVoxel(A.RemoveNans(raw[1]), voxel)
    prv = A.DownsampleVoxel(A.RemoveNans(raw[0]), voxel)
    ocur = O.downsample_voxel(O.remove_nans(raw[1]), voxel)
    oprv = O.downsample_voxel(O.remove_nans(raw[0]), voxel)
    assert np.array_equal(cur, ocur) and np.array_equal(prv, oprv)
    # 5 cm: above the replay's 8192 (k_sq_small); 10 cm: below it
    assert (8192 < len(cur) <= 16384) if voxel == 0.05 else (1000 < len(cur) <= 8192), len(cur)
    hctx = A.get_context()
    _enable_seq_trace(hctx, True)
    try:
        T = np.eye(4, dtype=np.float32)
        assert A.AlignIcp3d(cur, prv, 128, T)
        tr = _seq_trace(hctx, 128)
    finally:
        _enable_seq_trace(hctx, False)
    ok, To, mco, otr = O.align_icp(cur, prv, 128, trace=True, sum_mode=0)
    assert ok
    dmean = (tr[:, :3] / np.float32(len(cur))).astype(np.float32)
    assert np.array_equal(dmean.view(np.uint32), otr["dmean"].view(np.uint32))
    assert np.array_equal(tr[:, 3].view(np.uint32), otr["cost"].view(np.uint32))
    e = pose_err(T, To)
    print(f"callers' workload ({len(cur)} points): 128/128 iterations bit-exact, pose {e}")
    assert max(e) <= 1e-6, e
