"""CPU: the oracle against the golden vectors, the independent numpy
restatement, brute force and hand-checkable cases."""
from __future__ import annotations

import numpy as np
import pytest

import np_restate as NPR
from conftest import GOLDEN_NAMES, PAIR_NAMES, load_golden
from oracle import oracle as O
from posemetric import pose_err


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_oracle_reproduces_golden(name):
    g = load_golden(name)
    it = int(g["max_iter"])
    ok, T, mc, tr = O.align_icp(g["src"], g["dst"], it, trace=True)
    assert np.array_equal(tr["nn_idx0"], g["nn_idx0"])
    assert np.array_equal(tr["nn_d20"], g["nn_d20"])
    np.testing.assert_array_equal(tr["cov"][0], g["cov0"])
    np.testing.assert_array_equal(tr["cov"][1], g["cov1"])
    np.testing.assert_array_equal(tr["pose"][0], g["pose1"])
    np.testing.assert_array_equal(tr["pose"][7], g["pose8"])
    np.testing.assert_array_equal(T, g["pose_final"])
    assert ok == bool(g["ok"]) and np.float32(mc) == g["mean_cost"]
    _, T64, _, _ = O.align_icp(g["src"], g["dst"], it, sum_mode=1)
    np.testing.assert_array_equal(T64, g["pose_final_fp64"])


@pytest.mark.parametrize("name", ["random_128", "pair_80x60_s0"])
def test_numpy_restatement_matches_golden(name):
    g = load_golden(name)
    ok, T, mc, tr = NPR.align_icp(g["src"], g["dst"], int(g["max_iter"]), trace=True)
    assert np.array_equal(tr["nn_idx0"], g["nn_idx0"])
    assert np.array_equal(tr["nn_d20"], g["nn_d20"])
    np.testing.assert_allclose(tr["cov"][0], g["cov0"], rtol=1e-9, atol=1e-12)
    assert max(pose_err(T, g["pose_final"])) <= 2e-6


@pytest.mark.parametrize("name", ["random_128", "random_2048"])
def test_random_source_recovers_known_motion(name):
    """Identical point sets under a known rigid motion: the reference loop
    converges to it (to float precision)."""
    g = load_golden(name)
    ang, tr = pose_err(g["pose_final"], g["T_gt"])
    assert ang < 1e-6 and tr < 1e-6


def test_kdtree_equals_bruteforce_with_ties():
    rng = np.random.default_rng(0)
    # a lattice (massive exact ties) plus duplicated points plus noise
    g = np.stack(np.meshgrid(*[np.arange(8, dtype=np.float32) * 0.25] * 3), -1).reshape(-1, 3)
    dst = np.concatenate([g, g[:50], rng.normal(size=(300, 3)).astype(np.float32)])
    q = np.concatenate([g + 0.125, rng.normal(size=(500, 3)).astype(np.float32), g[:20]])
    t = O.KDTree(dst, 16)
    i1, d1 = t.query(q)
    i2, d2 = O.nn_bruteforce(dst, q)
    assert np.array_equal(i1, i2) and np.array_equal(d1, d2)
    # lowest index wins every tie
    for k in range(len(q)):
        dd = NPR.d2_ref(q[k][None], dst)
        assert i1[k] == np.nonzero(dd == dd.min())[0][0]


def test_knn_sorted_and_exact():
    rng = np.random.default_rng(1)
    dst = rng.uniform(-1, 1, size=(2000, 3)).astype(np.float32)
    q = rng.uniform(-1.2, 1.2, size=(200, 3)).astype(np.float32)
    idx, d2 = O.KDTree(dst).query(q, 16)
    for k in range(len(q)):
        dd = NPR.d2_ref(q[k][None], dst)
        order = np.lexsort((np.arange(len(dst)), dd))[:16]
        assert np.array_equal(idx[k], order) and np.array_equal(d2[k], dd[order])


def test_nonfinite_query_keeps_reference_outparams():
    dst = np.random.default_rng(2).normal(size=(100, 3)).astype(np.float32)
    q = np.array([[np.nan, 0, 0], [np.inf, 1, 1], [0, 0, 0]], np.float32)
    idx, d2 = O.KDTree(dst).query(q)
    assert idx[0] == 0 and d2[0] == np.finfo(np.float32).max
    assert idx[1] == 0 and d2[1] == np.finfo(np.float32).max
    assert d2[2] < 10


def test_centroid_is_fp32_sequential():
    rng = np.random.default_rng(3)
    c = rng.uniform(0, 5, size=(100003, 3)).astype(np.float32)
    np.testing.assert_array_equal(O.centroid(c), NPR.centroid(c))


def test_jacobi_svd_reconstructs():
    rng = np.random.default_rng(4)
    for _ in range(50):
        A = rng.normal(size=(3, 3)) * rng.uniform(1e-3, 1e4)
        U, S, V = O.jacobi_svd3(A)
        np.testing.assert_allclose(U @ np.diag(S) @ V.T, A, atol=1e-12 * np.abs(A).max() * 10)
        np.testing.assert_allclose(U.T @ U, np.eye(3), atol=1e-13)
        np.testing.assert_allclose(V.T @ V, np.eye(3), atol=1e-13)
        assert np.all(np.diff(S) <= 0)
        np.testing.assert_allclose(S, np.linalg.svd(A)[1], rtol=1e-12)


def test_kabsch_matches_numpy_restatement():
    rng = np.random.default_rng(5)
    for _ in range(50):
        cov = rng.normal(size=(3, 3)) * 100
        sm = rng.normal(size=3).astype(np.float32)
        dm = rng.normal(size=3).astype(np.float32)
        a = O.kabsch_pose(cov, sm, dm)
        b = NPR.kabsch_pose(cov, sm, dm)
        assert max(pose_err(a, b)) < 1e-6


def test_early_false_return_leaves_pose():
    T0 = np.diag([1, 1, 1, 1]).astype(np.float32)
    T0[0, 3] = 0.5
    ok, T, mc, _ = O.align_icp(np.zeros((2, 3), np.float32), np.zeros((10, 3), np.float32), 128, T0)
    assert not ok and np.array_equal(T, T0)
    ok, T, _, _ = O.align_icp(np.zeros((10, 3), np.float32), np.zeros((2, 3), np.float32), 128, T0)
    assert not ok and np.array_equal(T, T0)


def test_zero_iterations_is_identity_true():
    g = load_golden("random_128")
    ok, T, mc, _ = O.align_icp(g["src"], g["dst"], 0)
    assert ok and mc == 0.0 and np.array_equal(T, np.eye(4, dtype=np.float32))


def test_mu_schedule():
    g = load_golden("random_128")
    mu = g["mu"]
    exp = np.float32(1.0)
    for it in range(len(mu)):
        if it > 0 and it % 8 == 0:
            exp = np.float32(exp / np.float32(1.4))
        assert mu[it] == exp


@pytest.mark.parametrize("name", PAIR_NAMES)
def test_unproject_oracle_is_pinhole(name):
    g = load_golden(name)
    K4 = g["K4"]
    pts = O.unproject(g["depth_a"], K4)
    np.testing.assert_array_equal(pts, g["dst"])
    v, u = np.nonzero(g["depth_a"])
    z = np.float32(0.001) * g["depth_a"][v, u].astype(np.float32)
    x = ((u.astype(np.float32) - K4[2]) / K4[0]).astype(np.float32)
    np.testing.assert_array_equal(pts[:, 0], z * x)


@pytest.mark.parametrize("stride", [1, 2, 3, 4])
def test_unproject_strided_oracle_is_pinhole_subsample(stride):
    """Pyramid level (BASELINE configs[4]): the pixels (s*ul, s*vl), full
    intrinsics -- numpy restatement, and exactly a subset of level 0."""
    g = load_golden("pair_160x120_s2")
    K4 = g["K4"]
    d = g["depth_a"]
    pts = O.unproject(d, K4, stride=stride)
    v, u = np.nonzero(d[::stride, ::stride])
    v, u = v * stride, u * stride
    z = np.float32(0.001) * d[v, u].astype(np.float32)
    x = ((u.astype(np.float32) - K4[2]) / K4[0]).astype(np.float32)
    y = ((v.astype(np.float32) - K4[3]) / K4[1]).astype(np.float32)
    np.testing.assert_array_equal(pts, np.stack([z * x, z * y, z], 1))
    full = O.unproject(d, K4)
    keep = (np.nonzero(d.ravel())[0])
    sel = np.isin(keep, (v * d.shape[1] + u))
    np.testing.assert_array_equal(pts, full[sel])
    assert len(O.unproject(d, K4, keep_invalid=True, stride=stride)) == \
        d[::stride, ::stride].size


def test_pyramid_oracle_chain():
    g = load_golden("pair_160x120_s2")
    K4 = g["K4"]
    src = [O.unproject(g["depth_b"], K4, stride=1 << lv) for lv in range(3)]
    dst = [O.unproject(g["depth_a"], K4, stride=1 << lv) for lv in range(3)]
    # one level = AlignIcp3d
    ok1, T1, mc1 = O.align_icp_pyramid(src[:1], dst[:1], [16])
    ok, T, mc, _ = O.align_icp(src[0], dst[0], 16)
    assert ok1 == ok and np.array_equal(T1, T) and mc1 == mc
    # coarse-to-fine: the chain of calls with one pose
    okp, Tp, _ = O.align_icp_pyramid(src, dst, [16, 16, 32], sum_mode=1)
    Tc = np.eye(4, dtype=np.float32)
    for lv, it in ((2, 32), (1, 16), (0, 16)):
        _, Tc, _, _ = O.align_icp(src[lv], dst[lv], it, T=Tc, sum_mode=1)
    assert okp and np.array_equal(Tp, Tc)


@pytest.mark.parametrize("name", PAIR_NAMES)
def test_p2plane_oracle_converges_to_ground_truth(name):
    g = load_golden(name)
    ang, tr = pose_err(g["p2plane_pose"], g["T_gt"])
    assert ang < 2e-3 and tr < 3e-3, (ang, tr)
    assert 1 <= int(g["p2plane_iters"]) <= 30


def test_normals_oracle_unit_and_oriented():
    g = load_golden("pair_80x60_s0")
    n = g["normals_dst"]
    np.testing.assert_allclose(np.linalg.norm(n, axis=1), 1.0, atol=1e-5)
    assert np.all(np.sum(g["dst"] * n, axis=1) <= 0)  # face the viewpoint (origin)


def test_grid_normals_oracle_plane_and_golden_frames():
    """The image-grid normal restatement: a tilted plane's exact normal, and
    on the golden depth frames agreement with the kNN-16 normals."""
    h, w = 60, 80
    K4 = np.array([70.0, 70.0, 40.0, 30.0], np.float32)
    v, u = np.mgrid[0:h, 0:w].astype(np.float64)
    # plane z = 1.5 + 0.2 x  (x = (u - cx) / fx * z) -> solve z per pixel
    xr = (u - K4[2]) / K4[0]
    z = 1.5 / (1.0 - 0.2 * xr)
    depth = np.round(z * 1000).astype(np.uint16)
    n = O.grid_normals(depth, K4, 2)
    pts = O.unproject(depth, K4)
    assert n.shape == pts.shape
    true = np.array([0.2, 0.0, -1.0]) / np.linalg.norm([0.2, 0.0, -1.0])
    cos = n @ true
    assert np.median(cos) > 0.999, np.median(cos)
    np.testing.assert_allclose(np.linalg.norm(n, axis=1), 1.0, atol=1e-5)
    assert np.all(np.sum(pts * n, axis=1) <= 0)  # OrientNormals: face the camera
    for name in PAIR_NAMES:
        g = load_golden(name)
        gn = O.grid_normals(g["depth_a"], g["K4"], 2)
        assert gn.shape == g["normals_dst"].shape
        assert np.mean(np.sum(gn * g["normals_dst"], axis=1) > 0.9) > 0.9, name


def test_solve_kabsch_oracle_recovers_motion_and_matches_numpy():
    """SolveKabsch (align_icp.cpp:18-71): exact correspondences under a known
    rigid motion give that motion; weights enter the covariance linearly."""
    from realsensetracker_amd import driver
    rng = np.random.default_rng(7)
    src = rng.uniform(-1, 1, size=(500, 3)).astype(np.float32)
    D = driver.random_offset(rng, deg=(5.0, 10.0), cm=(5.0, 10.0))
    dst = (src.astype(np.float64) @ D[:3, :3].T + D[:3, 3]).astype(np.float32)
    perm = rng.permutation(500)
    dst_p = dst[perm]
    inv = np.argsort(perm)
    pairs = np.stack([np.arange(500), inv], 1)
    ok, T = O.solve_kabsch(src, dst_p, pairs)
    assert ok
    assert max(pose_err(T, D)) < 2e-6
    w = rng.uniform(0.1, 1.0, 500).astype(np.float32)
    ok, Tw = O.solve_kabsch(src, dst_p, pairs, w)
    assert ok and max(pose_err(Tw, D)) < 2e-6
    # the weighted covariance in numpy -> the same Kabsch
    sm = np.cumsum(src[pairs[:, 0]], 0, dtype=np.float32)[-1] / np.float32(500)
    dm = np.cumsum(dst_p[pairs[:, 1]], 0, dtype=np.float32)[-1] / np.float32(500)
    u = src[pairs[:, 0]] - sm
    v = dst_p[pairs[:, 1]] - dm
    cov = (w[:, None, None].astype(np.float64) *
           (v[:, :, None] * u[:, None, :]).astype(np.float64)).sum(0)
    Tn = O.kabsch_pose(cov, sm, dm)
    assert max(pose_err(Tw, Tn)) < 1e-6


def test_solve_kabsch_oracle_too_few_points():
    T0 = np.eye(4, dtype=np.float32)
    T0[0, 3] = 0.5
    ok, T = O.solve_kabsch(np.zeros((2, 3), np.float32), np.zeros((10, 3), np.float32),
                           [[0, 0], [1, 1]], T=T0)
    assert not ok and np.array_equal(T, T0)


# ---- f1: RemoveNans / DownsampleVoxel oracle vs the numpy restatement -------
import preproc_cases as PC  # noqa: E402


@pytest.mark.parametrize("name", sorted(PC.cases()))
def test_remove_nans_oracle_matches_numpy(name):
    cloud, _ = PC.cases()[name]
    np.testing.assert_array_equal(O.remove_nans(cloud), NPR.remove_nans(cloud))


@pytest.mark.parametrize("name", sorted(PC.cases()))
def test_downsample_voxel_oracle_matches_numpy(name):
    cloud, v = PC.cases()[name]
    got = O.downsample_voxel(cloud, v, order="input")
    np.testing.assert_array_equal(got, NPR.downsample_voxel(cloud, v))
    # one point per occupied voxel, each the first of its voxel
    k = NPR.voxel_keys(cloud, v)
    assert len(got) == (len(np.unique(k, axis=0)) if len(cloud) else 0)
    # the reference's order: the container's iteration over those points
    ref = O.downsample_voxel(cloud, v)
    keys = NPR.voxel_keys(got, v)
    np.testing.assert_array_equal(ref, got[NPR.umap_order_model(keys, O.umap_schedule(len(got)))])


def test_downsample_voxel_oracle_on_frame():
    cloud = PC.frame_cloud()
    got = O.downsample_voxel(cloud, PC.VOXEL, order="input")
    np.testing.assert_array_equal(got, NPR.downsample_voxel(cloud, PC.VOXEL))
    assert 0 < len(got) < len(cloud)
    ref = O.downsample_voxel(cloud, PC.VOXEL)
    assert not np.array_equal(ref, got)  # (the container's order is not the input's)
    np.testing.assert_array_equal(np.sort(ref.view(np.uint32).reshape(-1, 3), axis=0),
                                  np.sort(got.view(np.uint32).reshape(-1, 3), axis=0))


# ---- the reference's std::unordered_map order (rst_oracle_umap.cpp) ----------
@pytest.mark.parametrize("n", [0, 1, 2, 13, 14, 29, 30, 59, 60, 127, 1000, 4099, 20000, 70000])
def test_umap_order_model_matches_the_real_container(n):
    """The level model (np_restate.umap_order_model: what voxel.hip's
    k_umap_order computes) reproduces a real libstdc++ std::unordered_map's
    iteration order with the classic boost::hash_combine, across every
    rehash up to n -- negative, zero and INT_MIN coordinates included."""
    rng = np.random.default_rng(n)
    k = rng.integers(-40, 40, size=(3 * n + 64, 3)).astype(np.int32)
    k[::7, 1] = np.iinfo(np.int32).min
    k[::11] = 0
    _, first = np.unique(k, axis=0, return_index=True)
    k = k[np.sort(first)][:n]
    assert len(k) == n
    sch = O.umap_schedule(n)
    np.testing.assert_array_equal(O.umap_order(k), NPR.umap_order_model(k, sch))


def test_umap_schedule_of_the_library_matches_the_container():
    """voxel.hip's rehash schedule (libstdc++'s _Prime_rehash_policy, host
    code, rst_debug_umap_schedule) equals the bucket counts a real
    std::unordered_map goes through (no GPU call)."""
    import ctypes as C
    from realsensetracker_amd import _lib as L
    f = L.lib().rst_debug_umap_schedule
    f.restype = C.c_int
    f.argtypes = [C.c_int64, C.POINTER(C.c_int64), C.c_int64, C.POINTER(C.c_int64)]
    for n in [0, 1, 13, 14, 29, 30, 1000, 123457, 2000000]:
        out = np.zeros(256, np.int64)
        cnt = C.c_int64(0)
        assert f(n, out.ctypes.data_as(C.POINTER(C.c_int64)), 128, C.byref(cnt)) == 0
        got = [tuple(int(v) for v in out[2 * j:2 * j + 2]) for j in range(cnt.value)]
        assert got == O.umap_schedule(n), n


# ---- f2: GICP oracle (point_cloud_utils.cpp:100-161, align_gicp.cpp:41-163) ----
def _gicp_pair():
    g = load_golden("pair_160x120_s2")
    return (O.downsample_voxel(g["src"], 0.1), O.downsample_voxel(g["dst"], 0.1), g["T_gt"])


def test_covariances_oracle_matches_numpy():
    from scipy.spatial import cKDTree
    src, _, _ = _gicp_pair()
    cov = O.compute_covariances(src)
    _, ii = cKDTree(src.astype(np.float64)).query(src, 33)
    for k in range(0, len(src), max(1, len(src) // 50)):
        nb = src[ii[k, 1:]].astype(np.float64)
        c = nb - nb.mean(0)
        np.testing.assert_allclose(cov[k], c.T @ c / 31, rtol=1e-4, atol=1e-8)
    # use_gicp: eigenvalues (1, 1, 1e-2), the last along the smallest direction
    cg = O.compute_covariances(src, use_gicp=True)
    for k in range(0, len(src), max(1, len(src) // 20)):
        w = np.linalg.eigvalsh(cg[k].astype(np.float64))
        np.testing.assert_allclose(w, [1e-2, 1, 1], atol=1e-5)


def test_gicp_gradient_matches_finite_differences():
    src, dst, T = _gicp_pair()
    cs, cd = O.compute_covariances(src), O.compute_covariances(dst)
    idx, _ = O.KDTree(dst).query(src)

    def rod(w):
        th = np.linalg.norm(w)
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        if th < 1e-12:
            return np.eye(3) + K
        return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K

    # a pose near (not at) the optimum, so the gradient is well away from 0
    R = rod(np.array([0.01, -0.02, 0.005])) @ T[:3, :3].astype(np.float64)
    t = T[:3, 3].astype(np.float64) + 0.003

    F, H, g = O.gicp_eval(src, dst, cs, cd, idx, R, t)
    num = np.zeros(6)
    for k in range(6):
        dx = np.zeros(6)
        dx[k] = 1e-6
        fp = O.gicp_eval(src, dst, cs, cd, idx, rod(dx[:3]) @ R, t + dx[3:])[0]
        fm = O.gicp_eval(src, dst, cs, cd, idx, rod(-dx[:3]) @ R, t - dx[3:])[0]
        num[k] = (fp - fm) / 2e-6
    assert np.abs(g - num).max() <= 1e-4 * np.abs(num).max()
    assert np.all(np.linalg.eigvalsh(H) > 0)


def test_gicp_align_oracle_recovers_motion():
    src, dst, T = _gicp_pair()
    cost, P = O.gicp_align(src, dst)
    ang, tr = pose_err(P, T)
    assert ang < 1e-3 and tr < 3e-3, (ang, tr)
    assert np.isfinite(cost) and cost > 0


# ---- f4: CloudAccumulator oracle (rs_replay_app.cpp:76-129) -------------------
def _accum_numpy(clouds_poses, voxel):
    inv = np.float32(1.0 / voxel)
    seen, out = set(), []
    for T, cloud in clouds_poses:
        p = NPR.transform(T, cloud)
        with np.errstate(invalid="ignore", over="ignore"):
            q = p * inv
        ok = (q >= np.float32(-2147483648.0)) & (q < np.float32(2147483648.0))
        k = np.where(ok, np.trunc(np.where(ok, q, 0)), -2147483648).astype(np.int64)
        for i in range(len(p)):
            key = tuple(k[i])
            if key not in seen:
                seen.add(key)
                out.append(p[i])
    return np.array(out, np.float32).reshape(-1, 3)


def test_accumulator_oracle_matches_numpy():
    g = load_golden("pair_80x60_s0")
    rng = np.random.default_rng(5)
    T1 = np.eye(4, dtype=np.float32)
    T2 = g["T_gt"].astype(np.float32)
    extra = rng.uniform(-3, 3, (500, 3)).astype(np.float32)
    extra[:5] = np.nan
    seq = [(T1, g["src"]), (T2, g["dst"]), (T1, extra), (T2, g["src"])]
    acc = O.Accumulator(0.05)
    for T, c in seq:
        acc.add(T, c)
    ins = _accum_numpy(seq, 0.05)
    np.testing.assert_array_equal(acc.extract(order="input"), ins)
    # ExtractPointCloud (:112-121): the container's iteration order
    keys = O.vox_keys(ins, 0.05, 1)
    np.testing.assert_array_equal(acc.extract(), ins[NPR.umap_order_model(keys, O.umap_schedule(len(ins)))])


# ---- f3: FPFH oracle (fpfh.cpp:20-165,248-300) ----------------------------------
def test_fpfh_oracle_histograms_and_matches():
    src, dst, _ = _gicp_pair()
    fs = O.compute_fpfh(src, radius=0.5)
    h = fs.reshape(-1, 3, 11)
    s = h.sum(-1)
    # every point has neighbours at 0.5 m here: each histogram sums to 1
    np.testing.assert_allclose(s, 1.0, atol=1e-5)
    assert np.all(fs >= 0)
    fd = O.compute_fpfh(dst, radius=0.5)
    idx, d2 = O.compute_matches(fs, fd, 2)
    # brute force in float64 agrees on the nearest (no near-ties at this size)
    sub = fs[:200].astype(np.float64)
    full = ((sub[:, None, :] - fd[None, :, :].astype(np.float64)) ** 2).sum(-1)
    order = np.argsort(full, axis=1, kind="stable")[:, :2]
    agree = np.mean(order[:, 0] == idx[:200, 0])
    assert agree > 0.99
    assert np.all(d2[:, 0] <= d2[:, 1])
