"""A batch of frame pairs aligned in lockstep (rst_icp_align_batch_async,
icp.hip icp_launch_batch): one launch of each loop kernel for the whole
batch, every pair's result bit-identical to aligning it alone
(AlignIcp3d, align_icp.cpp:73-161) -- pose, mean cost, status -- in the
three modes; pairs with the reference's early false left out and
reported (:77-79)."""
import numpy as np
import pytest

from realsensetracker_amd import _lib as L
from realsensetracker_amd import align as A
from realsensetracker_amd import driver

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return A.get_context(0)


@pytest.fixture(scope="module")
def frames(ctx):
    K = driver.intrinsics(320, 240)
    sc = driver.SyntheticScene(2)
    deps = [sc.render(sc.trajectory(2 * k), K, noise_seed=k) for k in range(4)]
    return K, deps


def _targets(ctx, K, deps, normals_k=0):
    out = []
    for d in deps:
        b = A.DeviceBuffer.from_array(d, ctx)
        out.append(A.Target.from_depth_device(b.ptr, K, normals_k, ctx))
        ctx.synchronize()
        b.free()
    return out


@pytest.mark.parametrize("mode", ["ref", "fp64", "p2plane"])
def test_batch_equals_pairs_alone(ctx, frames, mode):
    K, deps = frames
    nk = -2 if mode == "p2plane" else 0
    t = _targets(ctx, K, deps, nk)
    if mode == "p2plane":
        opts = L.default_opts(mode=L.RST_P2PLANE, max_iter=30)
    else:
        opts = L.default_opts(max_iter=40, sum_mode=L.RST_SUM_REF if mode == "ref" else L.RST_SUM_FP64)
    tiny = A.Target.build(np.zeros((2, 3), np.float32), ctx)  # the reference's early false
    srcs = [t[1], t[2], tiny, t[3]]
    dsts = [t[0], t[1], t[2], t[2]]
    rng = np.random.default_rng(4)
    poses = []
    for k in range(4):
        P = np.eye(4, dtype=np.float32)
        P[:3, 3] = rng.normal(size=3).astype(np.float32) * 0.01
        poses.append(P)
    got = A.align_batch_async(srcs, dsts, ctx, poses, opts).wait()
    for k in range(4):
        if srcs[k] is tiny:
            assert not got[k].ok and np.array_equal(got[k].pose, poses[k])
            continue
        one = A.align_prepared_async(srcs[k], dsts[k], ctx, poses[k], opts).wait()
        assert got[k].ok == one.ok
        assert np.array_equal(got[k].pose, one.pose), (k, got[k].pose, one.pose)
        assert got[k].mean_cost == one.mean_cost
        assert got[k].iterations == one.iterations
    for x in t + [tiny]:
        x.free()


def test_batch_of_one_and_reuse(ctx, frames):
    K, deps = frames
    t = _targets(ctx, K, deps)
    opts = L.default_opts(max_iter=16, sum_mode=L.RST_SUM_REF)
    a = A.align_batch_async([t[1]], [t[0]], ctx, None, opts).wait()[0]
    one = A.align_prepared_async(t[1], t[0], ctx, None, opts).wait()
    assert np.array_equal(a.pose, one.pose) and a.mean_cost == one.mean_cost
    # a larger batch after a smaller one on the same context (state arrays grow)
    b = A.align_batch_async([t[1], t[2], t[3]], [t[0], t[1], t[2]], ctx, None, opts).wait()
    assert np.array_equal(b[0].pose, one.pose)
    for x in t:
        x.free()
