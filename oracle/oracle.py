"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker.  The product
(realsensetracker_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"

_f = C.POINTER(C.c_float)
_d = C.POINTER(C.c_double)
_i = C.POINTER(C.c_int32)
_u16 = C.POINTER(C.c_uint16)
_lib = None


class _Trace(C.Structure):
    _fields_ = [("pose", _f), ("cost", _f), ("mu", _f), ("cov", _d), ("dmean", _f),
                ("nn_idx0", _i), ("nn_d20", _f)]


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        P = C.c_void_p
        L.orc_kdtree_build.restype = P
        L.orc_kdtree_build.argtypes = [_f, C.c_int64, C.c_int]
        L.orc_kdtree_free.argtypes = [P]
        L.orc_kdtree_knn.argtypes = [P, _f, C.c_int, _i, _f]
        L.orc_nn_batch.argtypes = [P, _f, C.c_int64, _i, _f]
        L.orc_nn_bruteforce.argtypes = [_f, C.c_int64, _f, C.c_int64, _i, _f]
        L.orc_centroid.argtypes = [_f, C.c_int64, _f]
        L.orc_transform_points.argtypes = [_f, _f, C.c_int64, _f]
        L.orc_jacobi_svd3.argtypes = [_d, _d, _d, _d]
        L.orc_kabsch_pose.argtypes = [_d, _f, _f, _f]
        L.orc_solve_kabsch.restype = C.c_int
        L.orc_solve_kabsch.argtypes = [_f, C.c_int64, _f, C.c_int64, _i, _f, C.c_int64, _f]
        L.orc_align_icp.restype = C.c_int
        L.orc_align_icp.argtypes = [_f, C.c_int64, _f, C.c_int64, P, C.c_int, _f, _f,
                                    C.POINTER(_Trace)]
        L.orc_align_icp_ex.restype = C.c_int
        L.orc_align_icp_ex.argtypes = [_f, C.c_int64, _f, C.c_int64, P, C.c_int, _f, _f,
                                       C.POINTER(_Trace), C.c_int]
        L.orc_p2point_partials.argtypes = [_f, C.c_int64, P, _f, _f, _f, C.c_float, _d]
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_compute_normals.argtypes = [_f, C.c_int64, P, C.c_int, _f, _f]
        L.orc_unproject.restype = C.c_int64
        L.orc_unproject_strided.restype = C.c_int64
        L.orc_grid_normals.restype = C.c_int64
        L.orc_grid_normals.argtypes = [_u16, C.c_int, C.c_int, C.c_int, _f, C.c_float, C.c_int,
                                       _f, _f]
        L.orc_remove_nans.argtypes = [_f, C.c_int64, _f]
        L.orc_remove_nans.restype = C.c_int64
        L.orc_downsample_voxel.argtypes = [_f, C.c_int64, C.c_float, _f]
        L.orc_downsample_voxel.restype = C.c_int64
        L.orc_compute_covariances.argtypes = [_f, C.c_int64, P, C.c_int, _f]
        L.orc_gicp_eval.restype = C.c_double
        L.orc_gicp_eval.argtypes = [_f, C.c_int64, _f, _f, _f, _i, _d, _d, _d, _d]
        L.orc_gicp_solve.restype = C.c_double
        L.orc_gicp_solve.argtypes = [_f, C.c_int64, _f, _f, _f, _i, _f, C.c_int, _f,
                                     C.POINTER(C.c_int)]
        L.orc_gicp_align.restype = C.c_double
        L.orc_gicp_align.argtypes = [_f, C.c_int64, _f, C.c_int64, C.c_int, C.c_int, _f]
        L.orc_compute_fpfh.argtypes = [_f, C.c_int64, _f, C.c_int, C.c_float, _f]
        L.orc_compute_matches.argtypes = [_f, C.c_int64, _f, C.c_int64, C.c_int, _i, _f]
        L.orc_accum_create.restype = P
        L.orc_accum_create.argtypes = [C.c_float]
        L.orc_accum_free.argtypes = [P]
        L.orc_accum_add.argtypes = [P, _f, _f, C.c_int64]
        L.orc_accum_extract.restype = C.c_int64
        L.orc_accum_extract.argtypes = [P, _f]
        L.orc_umap_order.argtypes = [_i, C.c_int64, C.POINTER(C.c_int64)]
        L.orc_umap_schedule.restype = C.c_int64
        L.orc_umap_schedule.argtypes = [C.c_int64, C.POINTER(C.c_int64), C.c_int64]
        L.orc_unproject.argtypes = [_u16, C.c_int, C.c_int, _f, C.c_float, C.c_int, _f]
        L.orc_unproject_strided.argtypes = [_u16, C.c_int, C.c_int, C.c_int, _f, C.c_float,
                                            C.c_int, _f]
        L.orc_align_p2plane.restype = C.c_int
        L.orc_align_p2plane.argtypes = [_f, C.c_int64, _f, _f, C.c_int64, P, C.c_int,
                                        C.c_float, C.c_float, C.c_float, _f, _f]
        L.orc_p2plane_partials.argtypes = [_f, C.c_int64, P, _f, _f, _d, _d, C.c_float,
                                           C.c_float, _d]
        L.orc_p2plane_update.restype = C.c_int
        L.orc_p2plane_update.argtypes = [_d, _d, _d, _d, _d]
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(_f)


def _cloud(x):
    a = np.ascontiguousarray(np.asarray(x, np.float32))
    assert a.ndim == 2 and a.shape[1] == 3
    return a


def _cm(T):
    return np.ascontiguousarray(np.asarray(T, np.float32).reshape(4, 4).T).reshape(16).copy()


def _uncm(b):
    return np.asarray(b, np.float32).reshape(4, 4).T.copy()


class KDTree:
    def __init__(self, cloud, leaf: int = 16):
        self.cloud = _cloud(cloud)  # the tree references it (kdtree.hpp:30)
        self.h = lib().orc_kdtree_build(_fp(self.cloud), self.cloud.shape[0], leaf)

    def query(self, q, k: int = 1):
        q = _cloud(q)
        n = q.shape[0]
        if k == 1:
            idx = np.zeros(n, np.int32)
            d2 = np.zeros(n, np.float32)
            lib().orc_nn_batch(self.h, _fp(q), n, idx.ctypes.data_as(_i), _fp(d2))
            return idx, d2
        idx = np.zeros((n, k), np.int32)
        d2 = np.zeros((n, k), np.float32)
        for i in range(n):
            lib().orc_kdtree_knn(self.h, _fp(q[i]), k, idx[i].ctypes.data_as(_i), _fp(d2[i]))
        return idx, d2

    def __del__(self):
        try:
            lib().orc_kdtree_free(self.h)
        except Exception:
            pass


def nn_bruteforce(dst, q):
    dst, q = _cloud(dst), _cloud(q)
    idx = np.zeros(q.shape[0], np.int32)
    d2 = np.zeros(q.shape[0], np.float32)
    lib().orc_nn_bruteforce(_fp(dst), dst.shape[0], _fp(q), q.shape[0],
                            idx.ctypes.data_as(_i), _fp(d2))
    return idx, d2


def centroid(cloud):
    a = _cloud(cloud)
    out = np.zeros(3, np.float32)
    lib().orc_centroid(_fp(a), a.shape[0], _fp(out))
    return out


def transform_points(T, cloud):
    a = _cloud(cloud)
    out = np.zeros_like(a)
    lib().orc_transform_points(_fp(_cm(T)), _fp(a), a.shape[0], _fp(out))
    return out


def jacobi_svd3(A):
    a = np.ascontiguousarray(np.asarray(A, np.float64).T).reshape(9)
    u = np.zeros(9)
    s = np.zeros(3)
    v = np.zeros(9)
    lib().orc_jacobi_svd3(a.ctypes.data_as(_d), u.ctypes.data_as(_d), s.ctypes.data_as(_d),
                          v.ctypes.data_as(_d))
    return u.reshape(3, 3).T, s, v.reshape(3, 3).T


def kabsch_pose(cov, smean, dmean):
    c = np.ascontiguousarray(np.asarray(cov, np.float64).T).reshape(9)
    out = np.zeros(16, np.float32)
    lib().orc_kabsch_pose(c.ctypes.data_as(_d), _fp(np.asarray(smean, np.float32)),
                          _fp(np.asarray(dmean, np.float32)), _fp(out))
    return _uncm(out)


def solve_kabsch(src, dst, pairs, weights=None, T=None):
    """SolveKabsch (align_icp.cpp:18-71).  pairs: (k, 2) int (src, dst).
    Returns (ok, pose); pose = T (untouched) when ok is False."""
    src, dst = _cloud(src), _cloud(dst)
    p = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(-1, 2))
    w = None if weights is None else np.ascontiguousarray(np.asarray(weights, np.float32))
    T0 = np.eye(4, dtype=np.float32) if T is None else np.asarray(T, np.float32)
    out = _cm(T0)
    ok = lib().orc_solve_kabsch(_fp(src), len(src), _fp(dst), len(dst), p.ctypes.data_as(_i),
                                None if w is None else _fp(w), len(p), _fp(out))
    return bool(ok), _uncm(out)


def set_threads(k: int) -> None:
    """OpenMP threads of the NN loop (1 = the reference's single thread)."""
    lib().orc_set_threads(int(k))


def align_icp(src, dst, max_iter=128, T=None, tree: KDTree | None = None, trace=False,
              sum_mode: int = 0):
    """AlignIcp3d restatement.  Returns (ok, pose, mean_cost, trace-dict|None).
    sum_mode 0 = the reference's fp32 sequential sums; 1 = fp64 sums (the
    GPU's reduction arithmetic)."""
    s, d = _cloud(src), _cloud(dst)
    buf = _cm(np.eye(4) if T is None else T)
    mc = C.c_float(0)
    tr = None
    trp = None
    if trace and max_iter > 0:
        tr = {"pose": np.zeros((max_iter, 16), np.float32), "cost": np.zeros(max_iter, np.float32),
              "mu": np.zeros(max_iter, np.float32), "cov": np.zeros((max_iter, 9), np.float64),
              "dmean": np.zeros((max_iter, 3), np.float32),
              "nn_idx0": np.zeros(s.shape[0], np.int32), "nn_d20": np.zeros(s.shape[0], np.float32)}
        t = _Trace(_fp(tr["pose"]), _fp(tr["cost"]), _fp(tr["mu"]),
                   tr["cov"].ctypes.data_as(_d), _fp(tr["dmean"]),
                   tr["nn_idx0"].ctypes.data_as(_i), _fp(tr["nn_d20"]))
        trp = C.byref(t)
    ok = lib().orc_align_icp_ex(_fp(s), s.shape[0], _fp(d), d.shape[0],
                                tree.h if tree is not None else None, max_iter, _fp(buf),
                                C.byref(mc), trp, int(sum_mode))
    if tr is not None:
        tr["pose"] = np.stack([_uncm(p) for p in tr["pose"]])
        tr["cov"] = np.stack([c.reshape(3, 3).T for c in tr["cov"]])
    return bool(ok), _uncm(buf), float(mc.value), tr


def p2point_partials(src, tree: KDTree, pose, smean, mu):
    s = _cloud(src)
    out = np.zeros(16)
    lib().orc_p2point_partials(_fp(s), s.shape[0], tree.h, _fp(tree.cloud), _fp(_cm(pose)),
                               _fp(np.asarray(smean, np.float32)), float(mu),
                               out.ctypes.data_as(_d))
    return out


def compute_normals(cloud, k=16, viewpoint=(0, 0, 0), tree: KDTree | None = None):
    a = _cloud(cloud)
    t = tree or KDTree(a, 16)
    out = np.zeros_like(a)
    lib().orc_compute_normals(_fp(a), a.shape[0], t.h, k, _fp(np.asarray(viewpoint, np.float32)),
                              _fp(out))
    return out


def unproject(depth, K4, depth_scale=0.001, keep_invalid=False, stride=1):
    """Pinhole deprojection; stride > 1 = pyramid level (every stride-th
    pixel of every stride-th row, full-image intrinsics)."""
    d = np.ascontiguousarray(depth, np.uint16)
    h, w = d.shape
    out = np.zeros((h * w, 3), np.float32)
    n = lib().orc_unproject_strided(d.ctypes.data_as(_u16), w, h, int(stride),
                                    _fp(np.asarray(K4, np.float32)), C.c_float(depth_scale),
                                    int(keep_invalid), _fp(out))
    return out[:n].copy()


def grid_normals(depth, K4, radius=2, stride=1, viewpoint=(0, 0, 0), depth_scale=0.001):
    """Image-grid normals of the frame's level `stride` (k_grid_normals'
    restatement), in unproject order."""
    d = np.ascontiguousarray(depth, np.uint16)
    h, w = d.shape
    out = np.zeros((((h + stride - 1) // stride) * ((w + stride - 1) // stride), 3), np.float32)
    n = lib().orc_grid_normals(d.ctypes.data_as(_u16), w, h, int(stride),
                               _fp(np.asarray(K4, np.float32)), C.c_float(depth_scale),
                               int(radius), _fp(np.asarray(viewpoint, np.float32)), _fp(out))
    assert n >= 0
    return out[:n].copy()


def align_icp_pyramid(src_levels, dst_levels, iters, T=None, sum_mode: int = 0):
    """Coarse-to-fine chain of the AlignIcp3d restatement (BASELINE
    configs[4]; the reference has no pyramid): levels finest first, run
    coarsest first, one pose array passed through every level (a level's
    early false leaves it untouched).  Returns (ok, pose, mean_cost) of
    level 0."""
    T = np.eye(4, dtype=np.float32) if T is None else np.asarray(T, np.float32)
    ok, mc = False, 0.0
    for lv in reversed(range(len(src_levels))):
        ok, T, mc, _ = align_icp(src_levels[lv], dst_levels[lv], iters[lv], T=T,
                                 sum_mode=sum_mode)
    return ok, T, mc


def remove_nans(cloud):
    """RemoveNans (point_cloud_utils.cpp:163-174)."""
    a = _cloud(cloud)
    out = np.zeros_like(a)
    n = lib().orc_remove_nans(_fp(a), a.shape[0], _fp(out))
    return out[:n].copy()


def downsample_voxel(cloud, voxel_size, order: str = "reference"):
    """DownsampleVoxel (point_cloud_utils.cpp:34-68): the first point of each
    voxel, in the reference's std::unordered_map iteration order (:54-57;
    rst_oracle_umap.cpp), or order="input" for ascending input index."""
    a = _cloud(cloud)
    out = np.zeros_like(a)
    n = lib().orc_downsample_voxel(_fp(a), a.shape[0], float(voxel_size), _fp(out))
    out = out[:n].copy()
    if order == "input":
        return out
    return out[umap_order(vox_keys(out, voxel_size, 0))]


def vox_keys(points, voxel_size, kind: int):
    """The reference's voxel keys, int32 (n, 3): kind 0 DownsampleVoxel's
    (p / v).floor().cast<int>() (point_cloud_utils.cpp:41-42), kind 1
    CloudAccumulator's (p * float(1.0 / v)).cast<int>() (rs_replay_app.cpp:
    91-92,108-110); NaN / out of int range -> INT_MIN (x86-64 cvttss2si)."""
    a = _cloud(points)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        if kind == 0:
            q = np.floor(a / np.float32(voxel_size))
        else:
            q = np.trunc(a * np.float32(1.0 / float(voxel_size)))
        ok = (q >= np.float32(-2147483648.0)) & (q < np.float32(2147483648.0))
        return np.where(ok, np.where(ok, q, 0).astype(np.int64), np.iinfo(np.int32).min).astype(np.int32)


def umap_order(keys):
    """keys: (n, 3) int32, distinct, insertion order.  The insertion indices
    in the order a real std::unordered_map (this toolchain's libstdc++, the
    reference's classic boost::hash_combine) iterates them."""
    k = np.ascontiguousarray(np.asarray(keys, np.int32).reshape(-1, 3))
    out = np.zeros(len(k), np.int64)
    lib().orc_umap_order(k.ctypes.data_as(_i), len(k), out.ctypes.data_as(C.POINTER(C.c_int64)))
    return out


def umap_schedule(n: int):
    """(elements before the insert that rehashed, new bucket count) of a
    default-constructed std::unordered_map receiving n distinct keys."""
    cap = 128
    out = np.zeros(2 * cap, np.int64)
    k = lib().orc_umap_schedule(int(n), out.ctypes.data_as(C.POINTER(C.c_int64)), cap)
    assert k <= cap
    return [tuple(int(v) for v in out[2 * j:2 * j + 2]) for j in range(k)]


def compute_covariances(cloud, use_gicp=False, tree: KDTree | None = None):
    """ComputeCovariances (point_cloud_utils.cpp:100-161): (n, 3, 3) float32."""
    a = _cloud(cloud)
    t = tree or KDTree(a, 16)
    out = np.zeros((a.shape[0], 9), np.float32)
    lib().orc_compute_covariances(_fp(a), a.shape[0], t.h, int(use_gicp), _fp(out))
    return out.reshape(-1, 3, 3).transpose(0, 2, 1).copy()  # col-major -> (r, c)


def _covs_cm(covs):
    c = np.ascontiguousarray(np.asarray(covs, np.float32).transpose(0, 2, 1))
    return c.reshape(-1, 9)


def gicp_eval(src, dst, src_covs, dst_covs, idx, R, t):
    """(F, H (6x6), g (6)) of the GICP cost at (R, t) (fp64)."""
    s, d = _cloud(src), _cloud(dst)
    cs, cd = _covs_cm(src_covs), _covs_cm(dst_covs)
    ii = np.ascontiguousarray(idx, np.int32)
    Rr = np.ascontiguousarray(R, np.float64).reshape(9)
    tt = np.ascontiguousarray(t, np.float64).reshape(3)
    H = np.zeros(36)
    g = np.zeros(6)
    F = lib().orc_gicp_eval(_fp(s), s.shape[0], _fp(d), _fp(cs), _fp(cd), ii.ctypes.data_as(_i),
                            Rr.ctypes.data_as(_d), tt.ctypes.data_as(_d), H.ctypes.data_as(_d),
                            g.ctypes.data_as(_d))
    return F, H.reshape(6, 6), g


def gicp_solve(src, dst, src_covs, dst_covs, idx, seed=None, max_iter=64):
    """Inner ComputeAlignment (align_gicp.cpp:41-103): (cost, pose, evaluations)."""
    s, d = _cloud(src), _cloud(dst)
    cs, cd = _covs_cm(src_covs), _covs_cm(dst_covs)
    ii = np.ascontiguousarray(idx, np.int32)
    sd = _cm(np.eye(4) if seed is None else seed)
    out = np.zeros(16, np.float32)
    its = C.c_int(0)
    F = lib().orc_gicp_solve(_fp(s), s.shape[0], _fp(d), _fp(cs), _fp(cd), ii.ctypes.data_as(_i),
                             _fp(sd), max_iter, _fp(out), C.byref(its))
    return F, _uncm(out), its.value


def gicp_align(src, dst, outer_iters=16, max_inner=64):
    """ComputeAlignment(src, dst, &T) (align_gicp.cpp:105-163): (cost, pose)."""
    s, d = _cloud(src), _cloud(dst)
    out = np.zeros(16, np.float32)
    F = lib().orc_gicp_align(_fp(s), s.shape[0], _fp(d), d.shape[0], outer_iters, max_inner,
                             _fp(out))
    return F, _uncm(out)


def compute_fpfh(cloud, viewpoint=(0, 0, 0), normal_k=16, radius=0.5):
    """ComputeFpfh (fpfh.cpp:248-262): (n, 33) float32."""
    a = _cloud(cloud)
    out = np.zeros((a.shape[0], 33), np.float32)
    lib().orc_compute_fpfh(_fp(a), a.shape[0], _fp(np.asarray(viewpoint, np.float32)),
                           int(normal_k), float(radius), _fp(out))
    return out


def compute_matches(src_feat, dst_feat, k=2):
    """ComputeMatches (fpfh.cpp:285-300): (idx (n, k), d2 (n, k))."""
    s = np.ascontiguousarray(np.asarray(src_feat, np.float32).reshape(-1, 33))
    d = np.ascontiguousarray(np.asarray(dst_feat, np.float32).reshape(-1, 33))
    idx = np.zeros((len(s), k), np.int32)
    d2 = np.zeros((len(s), k), np.float32)
    lib().orc_compute_matches(_fp(s), len(s), _fp(d), len(d), int(k), idx.ctypes.data_as(_i),
                              _fp(d2))
    return idx, d2


class Accumulator:
    """CloudAccumulator (rs_replay_app.cpp:76-129)."""

    def __init__(self, voxel_size=0.05):
        self.voxel_size = float(voxel_size)
        self.h = lib().orc_accum_create(float(voxel_size))

    def add(self, T, cloud):
        a = _cloud(cloud)
        lib().orc_accum_add(self.h, _fp(_cm(T)), _fp(a), a.shape[0])

    def extract(self, order: str = "reference"):
        """ExtractPointCloud (rs_replay_app.cpp:112-121): the reference's
        std::unordered_map iteration order, or order="input" (insertion)."""
        n = lib().orc_accum_extract(self.h, None)
        out = np.zeros((n, 3), np.float32)
        lib().orc_accum_extract(self.h, _fp(out))
        if order == "input":
            return out
        return out[umap_order(vox_keys(out, self.voxel_size, 1))]

    def __del__(self):
        try:
            lib().orc_accum_free(self.h)
        except Exception:
            pass


def align_p2plane(src, dst, dst_normals, max_iter=30, eps=1e-6, mu=4e-4, max_dist=0.0, T=None,
                  tree: KDTree | None = None):
    s, d, nn = _cloud(src), _cloud(dst), _cloud(dst_normals)
    buf = _cm(np.eye(4) if T is None else T)
    mc = C.c_float(0)
    it = lib().orc_align_p2plane(_fp(s), s.shape[0], _fp(d), _fp(nn), d.shape[0],
                                 tree.h if tree is not None else None, max_iter, eps, mu,
                                 max_dist, _fp(buf), C.byref(mc))
    return it, _uncm(buf), float(mc.value)


def p2plane_partials(src, tree: KDTree, dst_normals, Rd, td, mu=4e-4, max_dist=0.0):
    """One point-to-plane iteration's normal equations over `src` (a shard)
    at the double pose (Rd 3x3, td 3): 29 doubles (21 lower-triangle sum
    w J J^T, 6 sum w J r, count, sum d2) -- orc_align_p2plane's own sums."""
    s, nn = _cloud(src), _cloud(dst_normals)
    out = np.zeros(29)
    R = np.ascontiguousarray(np.asarray(Rd, np.float64).T).reshape(9)
    t = np.ascontiguousarray(np.asarray(td, np.float64)).reshape(3)
    lib().orc_p2plane_partials(_fp(s), s.shape[0], tree.h, _fp(tree.cloud), _fp(nn),
                               R.ctypes.data_as(_d), t.ctypes.data_as(_d), float(mu),
                               float(max_dist), out.ctypes.data_as(_d))
    return out


def p2plane_update(tot, Rd, td):
    """The solve + pose update on the all-reduced sums.  Returns (ok, Rd, td,
    |xi|, cost)."""
    t_ = np.ascontiguousarray(np.asarray(tot, np.float64)).copy()
    R = np.ascontiguousarray(np.asarray(Rd, np.float64).T).reshape(9).copy()
    t = np.ascontiguousarray(np.asarray(td, np.float64)).reshape(3).copy()
    xn, cost = C.c_double(0), C.c_double(0)
    ok = lib().orc_p2plane_update(t_.ctypes.data_as(_d), R.ctypes.data_as(_d),
                                  t.ctypes.data_as(_d), C.byref(xn), C.byref(cost))
    return bool(ok), R.reshape(3, 3).T.copy(), t, xn.value, cost.value
