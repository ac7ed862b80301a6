"""Independent numpy/scipy restatement of AlignIcp3d (test infrastructure).

Written separately from oracle/rst_oracle.c to cross-check it:
  * NN through scipy.spatial.cKDTree (a different exact kd-tree), with the
    squared distance recomputed in float32 in nanoflann's op order and exact
    ties resolved to the lowest index by a brute-force re-check of every
    candidate within the float tolerance band;
  * fp32 sequential sums via np.cumsum(dtype=float32) (sequential by
    definition, unlike np.sum's pairwise reduction);
  * Kabsch via np.linalg.svd (LAPACK gesdd) instead of Eigen's JacobiSVD;
  * the quaternion round trip written from Eigen's formulas.
Reference: rs_tracker/align/src/align_icp.cpp:73-167,
rs_tracker/common/src/point_cloud_utils.cpp:92-98.
"""
from __future__ import annotations

import numpy as np
from scipy.spatial import cKDTree

f32 = np.float32


def seqsum(x: np.ndarray) -> np.float32:
    x = np.asarray(x, f32)
    return np.cumsum(x, dtype=f32)[-1] if len(x) else f32(0)


def centroid(cloud: np.ndarray) -> np.ndarray:
    """point_cloud_utils.cpp:92-98: fp32 sequential sum * float(1.0/n)."""
    n = len(cloud)
    s = np.array([seqsum(cloud[:, k]) for k in range(3)], f32)
    return (s * f32(1.0 / n)).astype(f32)


def transform(T: np.ndarray, s: np.ndarray) -> np.ndarray:
    """Isometry3f * v: t_r + (R_r0 s0 + (R_r1 s1 + R_r2 s2)), all fp32."""
    R = np.asarray(T, f32)[:3, :3]
    t = np.asarray(T, f32)[:3, 3]
    s = np.asarray(s, f32)
    out = np.empty_like(s)
    for r in range(3):
        a0 = R[r, 0] * s[:, 0]
        a1 = R[r, 1] * s[:, 1]
        a2 = R[r, 2] * s[:, 2]
        out[:, r] = t[r] + (a0 + (a1 + a2))
    return out


def d2_ref(q: np.ndarray, p: np.ndarray) -> np.ndarray:
    d = (np.asarray(q, f32) - np.asarray(p, f32)).astype(f32)
    r = d[..., 0] * d[..., 0]
    r = r + d[..., 1] * d[..., 1]
    r = r + d[..., 2] * d[..., 2]
    return r.astype(f32)


class NN:
    """Exact 1-NN with float32 nanoflann distances and lowest-index ties."""

    def __init__(self, dst: np.ndarray):
        self.dst = np.asarray(dst, f32)
        self.tree = cKDTree(self.dst.astype(np.float64))

    def query(self, q: np.ndarray, k_cand: int = 8):
        q = np.asarray(q, f32)
        k = min(k_cand, len(self.dst))
        dist, idx = self.tree.query(q.astype(np.float64), k=k)
        idx = np.asarray(idx).reshape(len(q), k)
        dist = np.asarray(dist).reshape(len(q), k)
        d2 = d2_ref(q[:, None, :], self.dst[idx])
        # lexicographic (d2, idx) minimum among candidates
        order = np.lexsort((idx, d2), axis=1)
        bi = idx[np.arange(len(q)), order[:, 0]]
        bd = d2[np.arange(len(q)), order[:, 0]]
        # if the k-th candidate could still tie/beat the float result, redo
        # that query by brute force (rare)
        unsure = dist[:, -1] ** 2 <= bd.astype(np.float64) * (1 + 1e-5) + 1e-12
        for i in np.nonzero(unsure)[0]:
            dd = d2_ref(q[i][None, :], self.dst)
            m = dd.min()
            bi[i] = int(np.nonzero(dd == m)[0][0])
            bd[i] = m
        return bi.astype(np.int32), bd.astype(f32)


def quat_roundtrip(R: np.ndarray) -> np.ndarray:
    """Quaternionf(R).toRotationMatrix() in fp32 (Eigen formulas)."""
    R = np.asarray(R, f32)
    q = np.zeros(4, f32)  # x y z w
    tr = (R[0, 0] + R[1, 1]) + R[2, 2]
    if tr > f32(0):
        t = np.sqrt(tr + f32(1))
        q[3] = f32(0.5) * t
        t = f32(0.5) / t
        q[0] = (R[2, 1] - R[1, 2]) * t
        q[1] = (R[0, 2] - R[2, 0]) * t
        q[2] = (R[1, 0] - R[0, 1]) * t
    else:
        i = 0
        if R[1, 1] > R[0, 0]:
            i = 1
        if R[2, 2] > R[i, i]:
            i = 2
        j = (i + 1) % 3
        k = (j + 1) % 3
        t = np.sqrt(R[i, i] - R[j, j] - R[k, k] + f32(1))
        q[i] = f32(0.5) * t
        t = f32(0.5) / t
        q[3] = (R[k, j] - R[j, k]) * t
        q[j] = (R[j, i] + R[i, j]) * t
        q[k] = (R[k, i] + R[i, k]) * t
    x, y, z, w = (f32(v) for v in q)
    tx, ty, tz = f32(2) * x, f32(2) * y, f32(2) * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[f32(1) - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, f32(1) - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, f32(1) - (txx + tyy)]], f32)


def kabsch_pose(cov: np.ndarray, smean: np.ndarray, dmean: np.ndarray) -> np.ndarray:
    U, S, Vt = np.linalg.svd(np.asarray(cov, np.float64))
    R = (U @ Vt).astype(f32)
    if np.linalg.det(R.astype(np.float64)) < 0:
        R[:, 2] *= f32(-1)
    t = np.empty(3, f32)
    for r in range(3):
        t[r] = dmean[r] - (R[r, 0] * smean[0] + (R[r, 1] * smean[1] + R[r, 2] * smean[2]))
    T = np.eye(4, dtype=f32)
    T[:3, :3] = quat_roundtrip(R)
    T[:3, 3] = t
    return T


def align_icp(src, dst, max_iter=128, T=None, trace=False):
    """AlignIcp3d restated; returns (ok, pose, mean_cost, trace)."""
    src = np.asarray(src, f32)
    dst = np.asarray(dst, f32)
    n = len(src)
    if n < 3 or len(dst) < 3:
        return False, (np.eye(4, dtype=f32) if T is None else T), 0.0, None
    nn = NN(dst)
    xfm = np.eye(4, dtype=f32) if T is None else np.asarray(T, f32).copy()
    smean = centroid(src)
    mu = f32(1.0)
    cost = f32(0)
    tr = {"pose": [], "cost": [], "cov": [], "dmean": [], "nn_idx0": None, "nn_d20": None}
    for it in range(max_iter):
        if it > 0 and it % 8 == 0:
            mu = f32(mu / f32(1.4))
        p = transform(xfm, src)
        j, d2 = nn.query(p)
        if it == 0:
            tr["nn_idx0"], tr["nn_d20"] = j, d2
        cost = seqsum(d2)
        l = (mu / (d2 + mu)).astype(f32)
        w = (l * l).astype(f32)
        q = dst[j]
        dmean = np.array([seqsum(q[:, k]) for k in range(3)], f32) / f32(n)
        a = (w[:, None] * (q - dmean).astype(f32)).astype(f32)
        u = (src - smean).astype(f32)
        prod = (a[:, :, None] * u[:, None, :]).astype(f32).astype(np.float64)
        cov = np.cumsum(prod, axis=0)[-1] if n else np.zeros((3, 3))
        xfm = kabsch_pose(cov, smean, dmean)
        if trace:
            tr["pose"].append(xfm.copy())
            tr["cost"].append(cost)
            tr["cov"].append(cov)
            tr["dmean"].append(dmean)
    mc = float(np.sqrt(f32(cost) / f32(n)))
    return mc < 10000, xfm, mc, (tr if trace else None)


# ---- preprocessing (point_cloud_utils.cpp:34-68, 163-174) -------------------
def remove_nans(cloud: np.ndarray) -> np.ndarray:
    """RemoveNans: rows whose three coordinates are finite, order kept."""
    a = np.asarray(cloud, f32)
    return a[np.isfinite(a).all(axis=1)]


def voxel_keys(cloud: np.ndarray, voxel_size: float) -> np.ndarray:
    """(point / voxel_size).floor().cast<int>() per axis (float32 division);
    NaN / out-of-int-range -> INT_MIN, x86-64's cvttss2si result."""
    a = np.asarray(cloud, f32)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        q = np.floor(a / f32(voxel_size))
        ok = (q >= f32(-2147483648.0)) & (q < f32(2147483648.0))
        return np.where(ok, q, 0).astype(np.int64).astype(np.int32) * ok + \
            np.int32(np.iinfo(np.int32).min) * ~ok


def downsample_voxel(cloud: np.ndarray, voxel_size: float) -> np.ndarray:
    """DownsampleVoxel: the first point of each voxel, in ascending index
    (np.unique's return_index is the first occurrence)."""
    a = np.asarray(cloud, f32)
    if len(a) == 0:
        return a.reshape(0, 3)
    k = voxel_keys(a, voxel_size).astype(np.int32)
    _, first = np.unique(k, axis=0, return_index=True)
    return a[np.sort(first)]


def boost_classic_hash(keys: np.ndarray) -> np.ndarray:
    """seed = 0; per coordinate seed ^= size_t(k) + 0x9e3779b9 + (seed << 6)
    + (seed >> 2) -- MatrixHash (point_cloud_utils.cpp:13-22) and VoxelHash
    (rs_replay_app.cpp:78-84) with Boost <= 1.80's hash_combine, uint64."""
    k = np.asarray(keys, np.int32).reshape(-1, 3).astype(np.int64).view(np.uint64)
    seed = np.zeros(len(k), np.uint64)
    with np.errstate(over="ignore"):
        for c in range(3):
            seed ^= k[:, c] + np.uint64(0x9E3779B9) + (seed << np.uint64(6)) + (seed >> np.uint64(2))
    return seed


def umap_order_model(keys: np.ndarray, schedule) -> np.ndarray:
    """The iteration order of a libstdc++ std::unordered_map that received
    `keys` (distinct, in order), from its rehash schedule alone (the model
    voxel.hip's k_umap_order computes):  between rehashes the list is one run
    per bucket, a bucket created later first, inside a bucket the later
    arrival first (an insert into an empty bucket goes to the list's front,
    any other to its bucket's front); a rehash walks the old list and
    re-inserts each node the same way.  So at every level the order sorts
    by (bucket's creation, arrival), both descending, where arrival = the
    node's position in the list the rehash walked, or its insertion index for
    keys inserted after it."""
    h = boost_classic_hash(keys)
    n = len(h)
    pos = np.zeros(0, np.int64)
    for lvl, (r, B) in enumerate(schedule):
        nl = schedule[lvl + 1][0] if lvl + 1 < len(schedule) else n
        a = np.arange(nl, dtype=np.int64)
        a[:r] = pos[:r]
        b = (h[:nl] % np.uint64(B)).astype(np.int64)
        ctime = np.full(B, np.iinfo(np.int64).max)
        np.minimum.at(ctime, b, a)
        order = np.lexsort((-a, -ctime[b]))
        pos = np.empty(nl, np.int64)
        pos[order] = np.arange(nl)
    out = np.empty(n, np.int64)
    out[pos] = np.arange(n)
    return out
