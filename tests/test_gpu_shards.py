"""GPU: the shard decomposition of the ICP loop (the
north_star's data-parallel split of align_icp.cpp:105-136) and the larger
BASELINE configs.

One GPU here, so the RCCL all-reduce between ranks is emulated on the host:
rst_debug_icp_partials gives the vector a rank contributes (its shard's
exact NN + partial sums), rst_debug_icp_solve the solve every rank runs on
the all-reduced vector.  Checked: shard vectors sum to the whole source's
(fp64 reassociation only), a host-driven two-shard loop reproduces the
unsharded device loop, and the single-rank RCCL path at configs[3] size
(~1M points) equals the unsharded loop bit for bit.  configs[2] (1280x720)
runs against the fp64-sum oracle."""
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

_dP = C.POINTER(C.c_double)


def _fns():
    lib = L.lib()
    p = lib.rst_debug_icp_partials
    p.restype = C.c_int
    p.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, L.c_float_p, C.c_float,
                  L.c_float_p, C.c_int32, _dP, L.c_int32_p]
    s = lib.rst_debug_icp_solve
    s.restype = C.c_int
    s.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, _dP, L.c_float_p, L.c_float_p,
                  L.c_float_p, L.c_int32_p]
    return p, s


def partials(ctx, src, tgt, opts, pose, mu, smean, it):
    p, _ = _fns()
    out = np.zeros(32, np.float64)
    nv = C.c_int32()
    buf = L.pose_to_cm(pose)
    sm = np.ascontiguousarray(smean, np.float32)
    L.check(p(ctx.handle, src.handle, tgt.handle, C.byref(opts), L.fptr(buf), float(mu),
              L.fptr(sm), int(it), out.ctypes.data_as(_dP), C.byref(nv)), "icp_partials")
    return out[:nv.value]


def solve(ctx, opts, n_total, tot, smean, pose, mu, it):
    _, s = _fns()
    t = np.zeros(32, np.float64)
    t[:len(tot)] = tot
    buf = L.pose_to_cm(pose)
    m = C.c_float(mu)
    k = C.c_int32(it)
    sm = np.ascontiguousarray(smean, np.float32)
    L.check(s(ctx.handle, C.byref(opts), int(n_total), t.ctypes.data_as(_dP), L.fptr(sm),
              L.fptr(buf), C.byref(m), C.byref(k)), "icp_solve")
    return L.cm_to_pose(buf), m.value, k.value


def fp64_centroid(x):
    """The RST_SUM_FP64 centroid: the fp64 sum / n rounded to float (k_init_state)."""
    return (x.astype(np.float64).sum(0) / len(x)).astype(np.float32)


def fp64(**kw):
    return L.default_opts(sum_mode=L.RST_SUM_FP64, **kw)


def _pair(w, h, scene, seed):
    K = driver.intrinsics(w, h)
    sc = driver.SyntheticScene(scene)
    da, db, D = driver.make_pair(sc, K, seed=seed)
    return K, driver.unproject(da, K), driver.unproject(db, K), D


@pytest.fixture(scope="module")
def ctx():
    return A.get_context(0)


@pytest.fixture(scope="module")
def pair640(ctx):
    K, pa, pb, D = _pair(640, 480, 5, 21)
    return pa, pb, D, A.Target.build(pa, ctx)


def test_shard_partials_sum_to_the_whole(ctx, pair640):
    """Two shards' partial-sum vectors add up to the whole source's, for the
    cold (ball-tile) and the warm iterations and at two poses."""
    pa, pb, D, t = pair640
    h = len(pb) // 2
    s_all, s_a, s_b = (A.Target.build(x, ctx) for x in (pb, pb[:h], pb[h:]))
    o = fp64()
    sm = fp64_centroid(pb)
    for pose in (np.eye(4, dtype=np.float32), D.astype(np.float32)):
        for it in (0, 40):
            full = partials(ctx, s_all, t, o, pose, o.mu0, sm, it)
            a = partials(ctx, s_a, t, o, pose, o.mu0, sm, it)
            b = partials(ctx, s_b, t, o, pose, o.mu0, sm, it)
            assert full.shape == (16,)
            scale = np.maximum(np.abs(full), 1e-12)
            assert np.all(np.abs(a + b - full) <= 1e-9 * scale + 1e-12), (it, a + b - full)


def test_shard_partials_p2plane(ctx, pair640):
    pa, pb, D, _ = pair640
    t = A.Target.build(pa, ctx)
    t.compute_normals(16)
    h = len(pb) // 3
    shards = [pb[:h], pb[h:2 * h], pb[2 * h:]]
    o = L.default_opts(mode=L.RST_P2PLANE)
    sm = np.zeros(3, np.float32)
    full = partials(ctx, A.Target.build(pb, ctx), t, o, np.eye(4, dtype=np.float32), o.mu0, sm, 0)
    parts = [partials(ctx, A.Target.build(x, ctx), t, o, np.eye(4, dtype=np.float32), o.mu0, sm,
                      0) for x in shards]
    assert full.shape == (30,)
    tot = np.sum(parts, axis=0)
    assert np.all(np.abs(tot - full) <= 1e-9 * np.maximum(np.abs(full), 1e-12) + 1e-12)


def _host_two_shard_loop(ctx, src, tgt, iters, o):
    h = len(src) // 2
    sa, sb = A.Target.build(src[:h], ctx), A.Target.build(src[h:], ctx)
    sm = fp64_centroid(src)  # the all-reduced centroid (fp64 sums)
    pose, mu, it = np.eye(4, dtype=np.float32), o.mu0, 0
    for _ in range(iters):
        tot = partials(ctx, sa, tgt, o, pose, mu, sm, it) + partials(ctx, sb, tgt, o, pose, mu, sm, it)
        pose, mu, it = solve(ctx, o, len(src), tot, sm, pose, mu, it)
    return pose, it


def test_host_emulated_two_shard_loop_640(ctx, pair640):
    """The sharded loop with its all-reduce on the host (two shards, 128
    iterations) against the unsharded device loop and the fp64-sum oracle."""
    pa, pb, D, t = pair640
    o = fp64(max_iter=128)
    pose, it = _host_two_shard_loop(ctx, pb, t, 128, o)
    assert it == 128
    r = A.align(pb, t, None, o)
    e = pose_err(pose, r.pose)
    print(f"host 2-shard loop vs unsharded: {e}")
    assert max(e) <= 2e-6, e
    _, To, _, _ = O.align_icp(pb, pa, 128, sum_mode=1)
    assert max(pose_err(pose, To)) <= 2e-5


def test_configs3_1M_shards(ctx):
    """BASELINE configs[3] size (1000x1000, ~1M points): the host-emulated
    two-shard loop, and the single-rank RCCL path bit-identical to the
    unsharded loop."""
    K, pa, pb, D = _pair(1000, 1000, 2, 7)
    assert len(pb) > 900_000
    t = A.Target.build(pa, ctx)
    o = fp64(max_iter=16)
    pose, _ = _host_two_shard_loop(ctx, pb, t, 16, o)
    r = A.align(pb, t, None, o)
    assert max(pose_err(pose, r.pose)) <= 2e-6
    uid = C.create_string_buffer(L.COMM_ID_BYTES)
    L.check(L.lib().rst_comm_get_unique_id(uid), "uid")
    comm = C.c_void_p()
    L.check(L.lib().rst_comm_create(ctx.handle, uid, 1, 0, C.byref(comm)), "comm")
    try:
        ds = A.DeviceBuffer.from_array(pb, ctx)
        buf = L.pose_to_cm(np.eye(4))
        mc = C.c_float(0)
        L.check(L.lib().rst_icp_align_sharded_device(ctx.handle, comm, C.c_void_p(ds.ptr), len(pb),
                                                     t.handle, C.byref(o), L.fptr(buf),
                                                     C.byref(mc)), "sharded")
        assert np.array_equal(L.cm_to_pose(buf), r.pose)
        # the reference-rounding mode sharded (correspondence all-gather,
        # sequential sums over the whole source, covariance all-reduce)
        oref = L.default_opts(max_iter=16, sum_mode=L.RST_SUM_REF)
        rr = A.align(pb, t, None, oref)
        buf = L.pose_to_cm(np.eye(4))
        L.check(L.lib().rst_icp_align_sharded_device(ctx.handle, comm, C.c_void_p(ds.ptr), len(pb),
                                                     t.handle, C.byref(oref), L.fptr(buf),
                                                     C.byref(mc)), "sharded ref")
        assert np.array_equal(L.cm_to_pose(buf), rr.pose)
    finally:
        L.lib().rst_comm_destroy(comm)


def _comm1(ctx):
    uid = C.create_string_buffer(L.COMM_ID_BYTES)
    L.check(L.lib().rst_comm_get_unique_id(uid), "uid")
    comm = C.c_void_p()
    L.check(L.lib().rst_comm_create(ctx.handle, uid, 1, 0, C.byref(comm)), "comm")
    return comm


def _sharded(ctx, comm, src, tgt, o):
    """rst_icp_align_sharded_device over one rank's shard (here: all of it)."""
    ds = A.DeviceBuffer.from_array(np.ascontiguousarray(src, np.float32), ctx)
    try:
        buf = L.pose_to_cm(np.eye(4))
        mc = C.c_float(0)
        st = L.check(L.lib().rst_icp_align_sharded_device(ctx.handle, comm, C.c_void_p(ds.ptr), len(src),
                                                          tgt.handle, C.byref(o), L.fptr(buf),
                                                          C.byref(mc)), "sharded")
        return st, L.cm_to_pose(buf), mc.value
    finally:
        ctx.synchronize()
        ds.free()


@pytest.mark.parametrize("size", ["640x480", "1000x1000"])
def test_sharded_p2plane_one_rank(ctx, size):
    """The north_star's multi-GPU path itself: point-to-plane with the
    source sharded and ONE RCCL all-reduce of the 6x6 / 6x1 normal equations
    (30 doubles) per iteration (rst_icp_align_sharded_device, icp.hip's comm
    branch: k_reduce_solve reduces only, ncclAllReduce, k_solve_only).  At
    one rank the all-reduce is an identity, so the pose, mean cost and status
    equal the unsharded loop's bit for bit -- at 640x480 and at configs[3]'s
    ~1M points -- and the pose is within 1e-6 of the C restatement's."""
    w, h = map(int, size.split("x"))
    K, pa, pb, D = _pair(w, h, 5 if w == 640 else 2, 21 if w == 640 else 7)
    t = A.Target.build(pa, ctx)
    t.compute_normals(16)
    o = L.default_opts(mode=L.RST_P2PLANE, max_iter=30)
    r = A.align(pb, t, None, o)
    assert r.ok
    comm = _comm1(ctx)
    try:
        st, pose, mc = _sharded(ctx, comm, pb, t, o)
        st2, pose2, _ = _sharded(ctx, comm, pb, t, o)  # cached layout, second align
    finally:
        L.lib().rst_comm_destroy(comm)
    assert st == L.RST_OK and st2 == L.RST_OK
    assert np.array_equal(pose, r.pose) and np.array_equal(pose2, r.pose), (pose, r.pose)
    assert np.float32(mc) == np.float32(r.mean_cost)
    if w == 640:
        nrm = t.normals()
        it, To, _ = O.align_p2plane(pb, pa, nrm, max_iter=30, eps=o.p2plane_eps, mu=o.p2plane_mu,
                                    max_dist=o.p2plane_max_dist, tree=O.KDTree(pa))
        e = pose_err(pose, To)
        print(f"sharded P2PLANE {size}: {r.iterations} vs {it} iterations, vs restatement {e}")
        assert max(e) <= 1e-6, e
    for x in (t,):
        x.free()


def test_sharded_p2plane_frame_target_640(ctx):
    """The same path on the bench's kind of target -- a 640x480 frame with
    image-grid normals, searched through its pixel windows.  A sharded align
    takes the narrow lone-pair window caps (kPixHalfLone), so its points
    split differently between the search kernels' fp64 partial-sum rows: the
    pose matches the unsharded loop and the C restatement to 1e-6, not bit
    for bit."""
    K = driver.intrinsics(640, 480)
    da, db, D = driver.make_pair(driver.SyntheticScene(5), K, seed=21)
    ba, bb = A.DeviceBuffer.from_array(da, ctx), A.DeviceBuffer.from_array(db, ctx)
    tf = A.Target.from_depth_device(ba.ptr, K, -2, ctx)
    sf = A.Target.from_depth_device(bb.ptr, K, 0, ctx)
    o = L.default_opts(mode=L.RST_P2PLANE, max_iter=30)
    r = A.align_prepared(sf, tf, None, o)
    pb = driver.unproject(db, K)
    comm = _comm1(ctx)
    try:
        st, pose, _ = _sharded(ctx, comm, pb, tf, o)
    finally:
        L.lib().rst_comm_destroy(comm)
    assert st == L.RST_OK and r.ok
    e = pose_err(pose, r.pose)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    pa = O.unproject(da, K4)
    it, To, _ = O.align_p2plane(O.unproject(db, K4), pa, tf.normals(), max_iter=30,
                                eps=o.p2plane_eps, mu=o.p2plane_mu, max_dist=o.p2plane_max_dist,
                                tree=O.KDTree(pa))
    eo = pose_err(pose, To)
    g = pose_err(pose, D)
    print(f"sharded P2PLANE frame target: vs unsharded {e}, vs restatement {eo}, vs truth {g}")
    assert max(e) <= 1e-6 and max(eo) <= 1e-6, (e, eo)
    for x in (tf, sf, ba, bb):
        x.free()


def test_sharded_seqsum_guard_is_an_error(ctx, pair640):
    """A tripped bound check of the sequential sums' tables inside the sharded
    REF relay (forced by rst_debug_seqsum_fault) is RST_E_HIP from the sharded
    align -- after comm_agree_guard has ORed every rank's guard word into every
    rank's, so all ranks fail the align together -- and the same
    communicator aligns normally once the hook is off."""
    from realsensetracker_amd.shard import ShardedAligner
    pa, pb, D, t = pair640
    f = L.lib().rst_debug_seqsum_fault
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_int32]
    sh = ShardedAligner(ctx, world=1, rank=0)
    ds = A.DeviceBuffer.from_array(pb, ctx)
    o = L.default_opts(max_iter=8, sum_mode=L.RST_SUM_REF)
    try:
        L.check(f(ctx.handle, 4), "rst_debug_seqsum_fault")
        try:
            with pytest.raises(L.RstError) as ei:
                sh.align(ds.ptr, len(pb), t, o, n_total=len(pb))
            assert "sequential-sum" in str(ei.value)
        finally:
            L.check(f(ctx.handle, 0), "rst_debug_seqsum_fault")
        ok, pose, _ = sh.align(ds.ptr, len(pb), t, o, n_total=len(pb))
        r = A.align(pb, t, None, o)
        assert ok and np.array_equal(pose, r.pose)
    finally:
        sh.close()
        ds.free()


def test_configs2_1280x720_tracks_oracle(ctx):
    """BASELINE configs[2] (1280x720, ~900k points): the device loop with
    fp64 sums against the fp64-sum oracle, and the NN at the final pose
    bit-exact on a sample of queries."""
    K, pa, pb, D = _pair(1280, 720, 3, 11)
    assert len(pb) > 800_000
    t = A.Target.build(pa, ctx)
    r = A.align(pb, t, None, fp64(max_iter=24))
    O.set_threads(8)
    try:
        _, To, _, _ = O.align_icp(pb, pa, 24, sum_mode=1)
    finally:
        O.set_threads(1)
    e = pose_err(r.pose, To)
    print(f"1280x720 vs fp64 oracle: {e}")
    assert max(e) <= 2e-5, e
    q = O.transform_points(r.pose, pb[:: max(1, len(pb) // 2000)])
    gi, gd = t.query(q)
    oi, od = O.nn_bruteforce(pa, q)
    assert np.array_equal(gi, oi) and np.array_equal(gd, od)
