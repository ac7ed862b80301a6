"""Host-side mirror of the reference's rs_tracker align / common API.

Same names, argument meaning and failure behaviour as
rs_tracker/align/include/rs_tracker/align/align_icp.hpp:14-24 and
rs_tracker/common/include/rs_tracker/common/point_cloud_utils.hpp:9-28, over
the MI355X C ABI (include/rst_align.h):

    AlignIcp3d(src, dst, max_iter, T)            -> bool  (T updated in place)
    AlignIcp3d(src, dst, dst_tree, max_iter, T)  -> bool
    KDTree3f(dst, leaf_max_size=16).query(p, k)  -> (indices, sq_dists)
    SolveKabsch(src, dst, indices, weights, T)   -> bool  (T updated in place)
    ComputeCentroid(cloud)                       -> (3,) float32
    ComputeNormals(cloud, tree, k)               -> (n, 3) float32
    OrientNormals(cloud, viewpoint, normals)     (in place)
    RemoveNans(cloud)                            -> (k, 3) float32
    DownsampleVoxel(cloud, voxel_size)           -> (k, 3) float32
    ComputeCovariances(tree, cloud, use_gicp)    -> (n, 3, 3) float32
    ComputeAlignment(src, dst, T) / (src, dst, src_covs, dst_covs, idx, seed, T)
                                                 -> cost (GICP; T updated)
    CloudAccumulator(voxel).AddCloud(xfm, cloud) / .ExtractPointCloud()
    ComputeFpfh(cloud, viewpoint, normal_k, radius) -> (n, 33) float32
    ComputeMatches(src_fpfh, dst_fpfh, 2)        -> (n, 2) int32
    PruneMatchesLowe(matches, src_fpfh, dst_fpfh, ratio) -> (pairs, weights)

Clouds are (n, 3) float32 arrays (the byte layout of Cloud3f); transforms are
4x4 float32 arrays in math orientation.
"""
from __future__ import annotations

import ctypes as C
import sys
from dataclasses import dataclass

import numpy as np

from . import _lib as L


class Context:
    """One GPU + one HIP stream (rst_ctx)."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        L.check(L.lib().rst_ctx_create(device, C.byref(self._h)), "rst_ctx_create")
        self.device = device

    @property
    def handle(self):
        return self._h

    def set_stream(self, hip_stream: int | None):
        L.check(L.lib().rst_ctx_set_stream(self._h, C.c_void_p(hip_stream or 0)),
                "rst_ctx_set_stream")

    def synchronize(self):
        L.check(L.lib().rst_ctx_synchronize(self._h), "rst_ctx_synchronize")

    def enable_kernel_timing(self, on: "bool | int" = True):
        """0/False off, 1/True every iteration, k > 1 every k-th."""
        L.check(L.lib().rst_ctx_enable_kernel_timing(self._h, int(on)), "timing")

    def enable_graphs(self, on: bool = True):
        """Replay each align's iteration loop as one hipGraph."""
        L.check(L.lib().rst_ctx_enable_graphs(self._h, int(on)), "rst_ctx_enable_graphs")

    def last_kernel_time(self):
        ms = C.c_float(0)
        n = C.c_int32(0)
        L.check(L.lib().rst_ctx_last_kernel_time(self._h, C.byref(ms), C.byref(n)), "timing")
        return ms.value, n.value

    def last_iteration_times(self):
        """Average ms per timed iteration: (kernel 1, kernel 2, the rest), n."""
        ms = np.zeros(3, np.float32)
        n = C.c_int32(0)
        L.check(L.lib().rst_ctx_last_iteration_times(self._h, L.fptr(ms), C.byref(n)), "timing")
        return [float(x) for x in ms], n.value

    def last_iterations(self) -> int:
        """Iterations run by the last align finished on this context."""
        n = C.c_int32(0)
        L.check(L.lib().rst_ctx_last_iterations(self._h, C.byref(n)), "rst_ctx_last_iterations")
        return n.value

    def close(self):
        if self._h:
            L.lib().rst_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        # no HIP calls while the interpreter tears down (objects die in
        # arbitrary order then; the OS reclaims the device memory)
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


_contexts: dict[int, Context] = {}


def get_context(device: int = 0) -> Context:
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]


class DeviceBuffer:
    """An HBM allocation through the library (rst_dev_alloc), for the
    *_device entry points: no second HIP runtime (torch's) in the process."""

    def __init__(self, nbytes: int, ctx: Context | None = None):
        self.ctx = ctx or get_context()
        self.nbytes = int(nbytes)
        self._p = C.c_void_p()
        L.check(L.lib().rst_dev_alloc(self.ctx.handle, self.nbytes, C.byref(self._p)),
                "rst_dev_alloc")

    @classmethod
    def from_array(cls, a: np.ndarray, ctx: Context | None = None) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, ctx)
        b.upload(a)
        return b

    @property
    def ptr(self) -> int:
        return self._p.value or 0

    def upload(self, a: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(a)
        if offset < 0 or offset + a.nbytes > self.nbytes:
            raise ValueError("upload past the buffer")
        L.check(L.lib().rst_dev_upload(self.ctx.handle, C.c_void_p(self.ptr + offset),
                                       a.ctypes.data_as(C.c_void_p), a.nbytes), "rst_dev_upload")

    def download(self, shape, dtype, offset: int = 0) -> np.ndarray:
        out = np.empty(shape, dtype)
        if offset < 0 or offset + out.nbytes > self.nbytes:
            raise ValueError("download past the buffer")
        L.check(L.lib().rst_dev_download(self.ctx.handle, out.ctypes.data_as(C.c_void_p),
                                         C.c_void_p(self.ptr + offset), out.nbytes),
                "rst_dev_download")
        return out

    def free(self) -> None:
        if self._p:
            L.lib().rst_dev_free(self.ctx.handle, self._p)
            self._p = C.c_void_p()

    def __del__(self):
        if sys.is_finalizing():
            return
        try:
            self.free()
        except Exception:
            pass


class Target:
    """Prepared target cloud in HBM: Morton-sorted points + exact-NN BVH
    (+ normals).  Replaces KDTree3f{dst, 16} (kdtree.hpp:27-57)."""

    def __init__(self, handle: C.c_void_p, ctx: Context):
        self._h = handle
        self.ctx = ctx

    @classmethod
    def build(cls, cloud, ctx: Context | None = None) -> "Target":
        ctx = ctx or get_context()
        a = L.as_cloud(cloud)
        h = C.c_void_p()
        L.check(L.lib().rst_target_build(ctx.handle, L.fptr(a), a.shape[0], C.byref(h)),
                "rst_target_build")
        return cls(h, ctx)

    @classmethod
    def build_device(cls, d_xyz_ptr: int, m: int, ctx: Context | None = None) -> "Target":
        ctx = ctx or get_context()
        h = C.c_void_p()
        L.check(L.lib().rst_target_build_device(ctx.handle, C.c_void_p(d_xyz_ptr), m,
                                                C.byref(h)), "rst_target_build_device")
        return cls(h, ctx)

    @classmethod
    def from_depth_device(cls, d_depth_ptr: int, K: "L.Intrinsics", normals_k: int = 0,
                          ctx: Context | None = None) -> "Target":
        ctx = ctx or get_context()
        h = C.c_void_p()
        L.check(L.lib().rst_frame_prepare_device(ctx.handle, C.c_void_p(d_depth_ptr),
                                                 C.byref(K), normals_k, C.byref(h)),
                "rst_frame_prepare_device")
        return cls(h, ctx)

    @classmethod
    def pyramid_from_depth_device(cls, d_depth_ptr: int, K: "L.Intrinsics", nlevels: int,
                                  normals_k: int = 0,
                                  ctx: Context | None = None) -> "list[Target]":
        """Targets of pyramid levels 0..nlevels-1 of one depth frame (level l:
        every 2^l-th pixel of every 2^l-th row, full-image intrinsics)."""
        ctx = ctx or get_context()
        hs = (C.c_void_p * nlevels)()
        L.check(L.lib().rst_frame_prepare_pyramid_device(ctx.handle, C.c_void_p(d_depth_ptr),
                                                         C.byref(K), nlevels, normals_k, hs),
                "rst_frame_prepare_pyramid_device")
        return [cls(C.c_void_p(hs[l]), ctx) for l in range(nlevels)]

    @property
    def handle(self):
        return self._h

    def __len__(self):
        return int(L.lib().rst_target_size(self._h))

    def query(self, points, num_closest: int = 1):
        """KDTree3f::query / knnSearch: exact k-NN, (idx, sq_dist) arrays."""
        q = L.as_cloud(points)
        n = q.shape[0]
        if num_closest == 1:
            idx = np.zeros(n, np.int32)
            d2 = np.zeros(n, np.float32)
            L.check(L.lib().rst_target_query_nn(self.ctx.handle, self._h, L.fptr(q), n,
                                                L.iptr(idx), L.fptr(d2)), "query_nn")
            return idx, d2
        idx = np.zeros((n, num_closest), np.int32)
        d2 = np.zeros((n, num_closest), np.float32)
        L.check(L.lib().rst_target_query_knn(self.ctx.handle, self._h, L.fptr(q), n,
                                             num_closest, L.iptr(idx), L.fptr(d2)), "query_knn")
        return idx, d2

    def query_warm(self, points, warm=None):
        """Exact 1-NN of a spatially coherent batch, optionally seeded with
        warm candidate indices (e.g. the previous frame's answer)."""
        q = L.as_cloud(points)
        n = q.shape[0]
        idx = np.zeros(n, np.int32)
        d2 = np.zeros(n, np.float32)
        w = None
        if warm is not None:
            w = np.ascontiguousarray(np.asarray(warm, np.int32))
            if w.shape != (n,):
                raise ValueError("warm must have one entry per query")
        L.check(L.lib().rst_target_query_nn_warm(self.ctx.handle, self._h, L.fptr(q), n,
                                                 L.iptr(w) if w is not None else None,
                                                 L.iptr(idx), L.fptr(d2)), "query_nn_warm")
        return idx, d2

    def compute_normals(self, k: int = 16, viewpoint=(0.0, 0.0, 0.0)):
        vp = np.asarray(viewpoint, np.float32)
        L.check(L.lib().rst_target_compute_normals(self.ctx.handle, self._h, k, L.fptr(vp)),
                "compute_normals")

    def compute_grid_normals(self, radius: int = 2, viewpoint=(0.0, 0.0, 0.0)):
        """Image-grid PCA normals over a (2 radius + 1)^2 pixel window (frame
        targets only: from_depth_device / pyramid_from_depth_device)."""
        vp = np.asarray(viewpoint, np.float32)
        L.check(L.lib().rst_target_compute_grid_normals(self.ctx.handle, self._h, radius,
                                                        L.fptr(vp)), "compute_grid_normals")

    def normals(self) -> np.ndarray:
        out = np.zeros((len(self), 3), np.float32)
        L.check(L.lib().rst_target_get_normals(self.ctx.handle, self._h, L.fptr(out)),
                "get_normals")
        return out

    def free(self):
        if self._h:
            L.lib().rst_target_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        if sys.is_finalizing():
            return
        try:
            self.free()
        except Exception:
            pass


class KDTree3f(Target):
    """Name-compatible constructor: KDTree3f(dst, leaf_max_size=16)."""

    def __init__(self, cloud, leaf_max_size: int = 16, ctx: Context | None = None):
        ctx = ctx or get_context()
        a = L.as_cloud(cloud)
        h = C.c_void_p()
        L.check(L.lib().rst_target_build(ctx.handle, L.fptr(a), a.shape[0], C.byref(h)),
                "rst_target_build")
        super().__init__(h, ctx)
        self.leaf_max_size = leaf_max_size


@dataclass
class IcpResult:
    ok: bool
    pose: np.ndarray
    mean_cost: float
    iterations: int


def align(src, target: Target, pose=None, opts: "L.IcpOpts | None" = None) -> IcpResult:
    """Full-result form of AlignIcp3d over a prepared target."""
    ctx = target.ctx
    s = L.as_cloud(src)
    pose = np.eye(4, dtype=np.float32) if pose is None else np.asarray(pose, np.float32)
    buf = L.pose_to_cm(pose)
    mc = C.c_float(0)
    o = opts if opts is not None else L.default_opts()
    st = L.check(L.lib().rst_icp_align(ctx.handle, L.fptr(s), s.shape[0], target.handle,
                                       C.byref(o), L.fptr(buf), C.byref(mc)), "rst_icp_align")
    return IcpResult(st == L.RST_OK, L.cm_to_pose(buf), float(mc.value), int(o.max_iter))


def align_prepared(src: Target, target: Target, pose=None,
                   opts: "L.IcpOpts | None" = None) -> IcpResult:
    pose = np.eye(4, dtype=np.float32) if pose is None else np.asarray(pose, np.float32)
    buf = L.pose_to_cm(pose)
    mc = C.c_float(0)
    it = C.c_int32(0)
    o = opts if opts is not None else L.default_opts()
    st = L.check(L.lib().rst_icp_align_prepared(target.ctx.handle, src.handle, target.handle,
                                                C.byref(o), L.fptr(buf), C.byref(mc),
                                                C.byref(it)), "rst_icp_align_prepared")
    return IcpResult(st == L.RST_OK, L.cm_to_pose(buf), float(mc.value), int(it.value))


class PendingAlign:
    """An align enqueued with align_prepared_async; .wait() -> IcpResult."""

    def __init__(self, ctx: Context, pose: np.ndarray, refs):
        self.ctx = ctx
        self._buf = L.pose_to_cm(pose)
        self._refs = refs  # src / target stay alive until wait()

    def wait(self) -> IcpResult:
        mc = C.c_float(0)
        it = C.c_int32(0)
        st = L.check(L.lib().rst_icp_align_wait(self.ctx.handle, L.fptr(self._buf), C.byref(mc),
                                                C.byref(it)), "rst_icp_align_wait")
        self._refs = None
        return IcpResult(st == L.RST_OK, L.cm_to_pose(self._buf), float(mc.value), int(it.value))


def align_prepared_async(src: Target, target: Target, ctx: Context, pose=None,
                         opts: "L.IcpOpts | None" = None) -> PendingAlign:
    """Enqueue AlignIcp3d(src, target) on ctx's stream and return at once;
    one pending align per context (use one context per frame pair in
    flight)."""
    pose = np.eye(4, dtype=np.float32) if pose is None else np.asarray(pose, np.float32)
    o = opts if opts is not None else L.default_opts()
    p = PendingAlign(ctx, pose, (src, target))
    L.check(L.lib().rst_icp_align_prepared_async(ctx.handle, src.handle, target.handle,
                                                 C.byref(o), L.fptr(L.pose_to_cm(pose))),
            "rst_icp_align_prepared_async")
    return p


class PendingBatch:
    """A batch enqueued with align_batch_async; .wait() -> [IcpResult]."""

    def __init__(self, ctx: Context, poses: np.ndarray, refs, nb: int):
        self.ctx = ctx
        self._buf = np.ascontiguousarray(np.stack([L.pose_to_cm(p) for p in poses]), np.float32)
        if len(self._buf) != nb:  # the C side reads and writes nb poses
            raise ValueError("one pose per pair")
        self._nb = nb
        self._refs = refs  # sources / targets stay alive until wait()

    def wait(self) -> list:
        nb = self._nb  # the count the C call was given: it writes nb of each
        mc = np.zeros(nb, np.float32)
        st = np.zeros(nb, np.int32)
        it = np.zeros(nb, np.int32)
        L.check(L.lib().rst_icp_align_batch_wait(self.ctx.handle, L.fptr(self._buf), L.fptr(mc),
                                                 st.ctypes.data_as(L.c_int32_p),
                                                 it.ctypes.data_as(L.c_int32_p)),
                "rst_icp_align_batch_wait")
        self._refs = None
        return [IcpResult(int(st[k]) == L.RST_OK, L.cm_to_pose(self._buf[k]), float(mc[k]), int(it[k]))
                for k in range(nb)]


def align_batch_async(srcs, targets, ctx: Context, poses=None,
                      opts: "L.IcpOpts | None" = None) -> PendingBatch:
    """Enqueue AlignIcp3d(srcs[k], targets[k]) for a batch of independent
    frame pairs on ctx's stream, in lockstep (rst_icp_align_batch_async):
    one launch per loop kernel for the whole batch, every result
    bit-identical to aligning the pair alone.  .wait() -> [IcpResult]."""
    nb = len(srcs)
    if len(targets) != nb or nb < 1:
        raise ValueError("srcs and targets need one entry per pair")
    poses = [np.eye(4, dtype=np.float32)] * nb if poses is None else [np.asarray(p, np.float32) for p in poses]
    if len(poses) != nb:
        raise ValueError("poses needs one 4x4 pose per pair")
    o = opts if opts is not None else L.default_opts()
    sh = (C.c_void_p * nb)(*[t.handle.value for t in srcs])
    th = (C.c_void_p * nb)(*[t.handle.value for t in targets])
    p = PendingBatch(ctx, poses, (list(srcs), list(targets)), nb)
    L.check(L.lib().rst_icp_align_batch_async(ctx.handle, nb, sh, th, C.byref(o), L.fptr(p._buf)),
            "rst_icp_align_batch_async")
    return p


def align_pyramid_async(src_levels, tgt_levels, ctx: Context, iters, pose=None,
                        opts: "L.IcpOpts | None" = None) -> PendingAlign:
    """Enqueue the coarse-to-fine ICP (rst_icp_align_pyramid_async): levels
    are finest first; runs coarsest -> finest, iters[l] iterations at level
    l, the pose chained on the device.  .wait() -> level 0's IcpResult."""
    nl = len(src_levels)
    if len(tgt_levels) != nl or len(iters) != nl or nl < 1:
        raise ValueError("src_levels, tgt_levels and iters need one entry per level")
    pose = np.eye(4, dtype=np.float32) if pose is None else np.asarray(pose, np.float32)
    o = opts if opts is not None else L.default_opts()
    sh = (C.c_void_p * nl)(*[t.handle.value for t in src_levels])
    th = (C.c_void_p * nl)(*[t.handle.value for t in tgt_levels])
    it = np.ascontiguousarray(iters, np.int32)
    p = PendingAlign(ctx, pose, (list(src_levels), list(tgt_levels)))
    L.check(L.lib().rst_icp_align_pyramid_async(ctx.handle, sh, th, nl,
                                                it.ctypes.data_as(L.c_int32_p), C.byref(o),
                                                L.fptr(L.pose_to_cm(pose))),
            "rst_icp_align_pyramid_async")
    return p


def align_pyramid(src_levels, tgt_levels, iters, pose=None,
                  opts: "L.IcpOpts | None" = None) -> IcpResult:
    """Blocking align_pyramid_async on the targets' context."""
    return align_pyramid_async(src_levels, tgt_levels, tgt_levels[0].ctx, iters, pose,
                               opts).wait()


def AlignIcp3d(src, dst, *args, opts: "L.IcpOpts | None" = None) -> bool:
    """AlignIcp3d(src, dst, max_iter, T) / AlignIcp3d(src, dst, dst_tree, max_iter, T).

    T (4x4 float32) is the in/out initial guess, left untouched on the early
    false return (align_icp.cpp:77-79); returns the reference's bool."""
    if len(args) == 2:
        tree, (max_iter, T) = None, args
    elif len(args) == 3:
        tree, max_iter, T = args
    else:
        raise TypeError("AlignIcp3d(src, dst, [dst_tree,] max_iter, transform)")
    if not (isinstance(T, np.ndarray) and T.shape == (4, 4) and T.dtype == np.float32):
        raise TypeError("transform must be a (4, 4) float32 ndarray (updated in place)")
    o = opts if opts is not None else L.default_opts()
    o.max_iter = int(max_iter)
    s = L.as_cloud(src)
    buf = L.pose_to_cm(T)
    mc = C.c_float(0)
    if tree is None:
        d = L.as_cloud(dst)
        ctx = get_context()
        st = L.check(L.lib().rst_icp_align_clouds(ctx.handle, L.fptr(s), s.shape[0], L.fptr(d),
                                                  d.shape[0], C.byref(o), L.fptr(buf),
                                                  C.byref(mc)), "rst_icp_align_clouds")
    else:
        st = L.check(L.lib().rst_icp_align(tree.ctx.handle, L.fptr(s), s.shape[0], tree.handle,
                                           C.byref(o), L.fptr(buf), C.byref(mc)),
                     "rst_icp_align")
    if len(s) >= 3 and len(dst) >= 3:
        T[...] = L.cm_to_pose(buf)
    return st == L.RST_OK


def SolveKabsch(src, dst, indices, weights, xfm: np.ndarray, ctx: Context | None = None) -> bool:
    """SolveKabsch(src, dst, indices, weights, &xfm) (align_icp.cpp:18-71) on the GPU.

    indices: (k, 2) int pairs (src index, dst index); weights: (k,) or
    empty/None for the unweighted branch.  xfm (4x4 float32) is written in
    place; untouched when the reference returns false (< 3 points)."""
    if not (isinstance(xfm, np.ndarray) and xfm.shape == (4, 4) and xfm.dtype == np.float32):
        raise TypeError("xfm must be a (4, 4) float32 ndarray (updated in place)")
    ctx = ctx or get_context()
    s, d = L.as_cloud(src), L.as_cloud(dst)
    p = np.ascontiguousarray(np.asarray(indices, np.int32).reshape(-1, 2))
    w = None
    if weights is not None and len(weights) > 0:
        w = np.ascontiguousarray(np.asarray(weights, np.float32))
        if len(w) != len(p):
            raise ValueError("weights must match indices")
    buf = L.pose_to_cm(xfm)
    st = L.check(L.lib().rst_solve_kabsch(ctx.handle, L.fptr(s), len(s), L.fptr(d), len(d),
                                          L.iptr(p), None if w is None else L.fptr(w), len(p),
                                          L.fptr(buf)), "rst_solve_kabsch")
    if st == L.RST_OK:
        xfm[...] = L.cm_to_pose(buf)
    return st == L.RST_OK


def ComputeCentroid(cloud, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or get_context()
    a = L.as_cloud(cloud)
    out = np.zeros(3, np.float32)
    L.check(L.lib().rst_compute_centroid(ctx.handle, L.fptr(a), a.shape[0], L.fptr(out)),
            "rst_compute_centroid")
    return out


def RemoveNans(cloud, ctx: Context | None = None) -> np.ndarray:
    """point_cloud_utils.cpp:163-174: the points with three finite
    coordinates, in input order."""
    ctx = ctx or get_context()
    a = L.as_cloud(cloud)
    out = np.zeros_like(a)
    n = C.c_int64(0)
    L.check(L.lib().rst_remove_nans(ctx.handle, L.fptr(a), a.shape[0], L.fptr(out), C.byref(n)),
            "rst_remove_nans")
    return out[:n.value].copy()


def DownsampleVoxel(cloud, voxel_size: float, ctx: Context | None = None) -> np.ndarray:
    """point_cloud_utils.cpp:34-68: the first point of every voxel
    floor(p / voxel_size), in the reference's order: its std::unordered_map's
    iteration (:54-57), replayed on the device (voxel.hip)."""
    ctx = ctx or get_context()
    a = L.as_cloud(cloud)
    out = np.zeros_like(a)
    n = C.c_int64(0)
    L.check(L.lib().rst_downsample_voxel(ctx.handle, L.fptr(a), a.shape[0], float(voxel_size),
                                         L.fptr(out), C.byref(n)), "rst_downsample_voxel")
    return out[:n.value].copy()


def ComputeFpfh(cloud, viewpoint=(0.0, 0.0, 0.0), normal_k: int = 16,
                feature_radius: float = 0.5, ctx: Context | None = None) -> np.ndarray:
    """fpfh.cpp:248-262: (n, 33) float32 FPFH features (rs_align_app's
    defaults: normal_k 16, radius 0.5)."""
    ctx = ctx or get_context()
    a = L.as_cloud(cloud)
    out = np.zeros((len(a), 33), np.float32)
    vp = np.asarray(viewpoint, np.float32)
    L.check(L.lib().rst_compute_fpfh(ctx.handle, L.fptr(a), len(a), L.fptr(vp), int(normal_k),
                                     float(feature_radius), L.fptr(out)), "rst_compute_fpfh")
    return out


def ComputeMatches(src_fpfh, dst_fpfh, num_matches: int = 2,
                   ctx: Context | None = None) -> np.ndarray:
    """fpfh.cpp:285-300: (n, num_matches) int32 indices of the nearest dst
    features (num_matches 1 or 2)."""
    ctx = ctx or get_context()
    s = np.ascontiguousarray(np.asarray(src_fpfh, np.float32).reshape(-1, 33))
    d = np.ascontiguousarray(np.asarray(dst_fpfh, np.float32).reshape(-1, 33))
    out = np.zeros((len(s), num_matches), np.int32)
    L.check(L.lib().rst_compute_matches(ctx.handle, L.fptr(s), len(s), L.fptr(d), len(d),
                                        int(num_matches), L.iptr(out), None),
            "rst_compute_matches")
    return out


def PruneMatchesLowe(matches, src_fpfh, dst_fpfh, lowe_ratio: float = 0.9):
    """rs_align_app.cpp:177-217 (the caller's host code): keep (i, j0) when
    d0 < lowe_ratio * d1 (or (i, j1) symmetrically), weight exp(-d / 0.0625)
    with d the squared feature distance.  Returns (pairs (k, 2) int32,
    weights (k,) float32)."""
    m = np.asarray(matches, np.int64)
    s = np.asarray(src_fpfh, np.float32)
    d = np.asarray(dst_fpfh, np.float32)
    r = np.float32(lowe_ratio)
    kvar = np.float32(0.25 * 0.25)
    pairs, w = [], []
    for i in range(len(m)):
        j0, j1 = int(m[i, 0]), int(m[i, 1])
        e0 = s[i] - d[j0]
        e1 = s[i] - d[j1]
        d0 = np.float32(np.sum(e0 * e0, dtype=np.float32))
        d1 = np.float32(np.sum(e1 * e1, dtype=np.float32))
        if d0 < d1:
            if d0 < r * d1:
                pairs.append((i, j0))
                w.append(np.exp(-d0 / kvar))
        elif d1 < r * d0:
            pairs.append((i, j1))
            w.append(np.exp(-d1 / kvar))
    return (np.asarray(pairs, np.int32).reshape(-1, 2), np.asarray(w, np.float32))


class CloudAccumulator:
    """rs_replay_app.cpp:76-129 on the device: AddCloud(xfm, cloud) keeps
    the first point (after xfm) of every voxel (int)(p / voxel_size);
    ExtractPointCloud() returns them in the reference's order, its
    std::unordered_map's iteration (:112-121)."""

    def __init__(self, voxel_size: float = 0.05, ctx: Context | None = None):
        self.ctx = ctx or get_context()
        self._h = C.c_void_p()
        L.check(L.lib().rst_accum_create(self.ctx.handle, float(voxel_size), C.byref(self._h)),
                "rst_accum_create")

    def AddCloud(self, xfm, cloud) -> None:
        a = L.as_cloud(cloud)
        L.check(L.lib().rst_accum_add(self._h, L.fptr(L.pose_to_cm(xfm)), L.fptr(a), len(a)),
                "rst_accum_add")

    def __len__(self) -> int:
        n = C.c_int64(0)
        L.check(L.lib().rst_accum_size(self._h, C.byref(n)), "rst_accum_size")
        return n.value

    def ExtractPointCloud(self) -> np.ndarray:
        out = np.zeros((len(self), 3), np.float32)
        n = C.c_int64(0)
        L.check(L.lib().rst_accum_extract(self._h, L.fptr(out), C.byref(n)), "rst_accum_extract")
        return out[:n.value]

    def __del__(self):
        if sys.is_finalizing():
            return
        try:
            if self._h:
                L.lib().rst_accum_destroy(self._h)
                self._h = C.c_void_p()
        except Exception:
            pass


def ComputeCovariances(tree: Target, cloud=None, use_gicp: bool = False) -> np.ndarray:
    """point_cloud_utils.cpp:100-161 on `tree`'s cloud (the reference passes
    the tree and the cloud it indexes; `cloud` is accepted for that shape and
    must be the same points): (m, 3, 3) float32 per point, original order."""
    m = len(tree)
    if cloud is not None and len(L.as_cloud(cloud)) != m:
        raise ValueError("cloud must be the tree's cloud")
    out = np.zeros((m, 9), np.float32)
    L.check(L.lib().rst_compute_covariances(tree.ctx.handle, tree.handle, int(bool(use_gicp)),
                                            L.fptr(out)), "rst_compute_covariances")
    return out.reshape(-1, 3, 3).transpose(0, 2, 1).copy()  # col-major -> [r, c]


def _covs_cm(covs) -> np.ndarray:
    c = np.asarray(covs, np.float32).reshape(-1, 3, 3)
    return np.ascontiguousarray(c.transpose(0, 2, 1)).reshape(-1, 9)


def ComputeAlignment(src, dst, *args, max_iter: int = 64, outer_iters: int = 16,
                     ctx: Context | None = None) -> float:
    """GICP (align_gicp.cpp): ComputeAlignment(src, dst, T) or
    ComputeAlignment(src, dst, src_covs, dst_covs, dst_indices, seed, T).
    T (4x4 float32) receives the result; returns the final cost (inf, T
    untouched, when the solve produced a non-finite pose)."""
    ctx = ctx or get_context()
    s, d = L.as_cloud(src), L.as_cloud(dst)
    cost = C.c_double(0.0)
    out = np.zeros(16, np.float32)
    if len(args) == 1:
        (T,) = args
        st = L.check(L.lib().rst_gicp_align(ctx.handle, L.fptr(s), len(s), L.fptr(d), len(d),
                                            int(outer_iters), int(max_iter), L.fptr(out),
                                            C.byref(cost)), "rst_gicp_align")
    elif len(args) == 5:
        src_covs, dst_covs, idx, seed, T = args
        cs, cd = _covs_cm(src_covs), _covs_cm(dst_covs)
        ii = np.ascontiguousarray(idx, np.int32)
        sd = L.pose_to_cm(seed)
        its = C.c_int32(0)
        st = L.check(L.lib().rst_gicp_solve(ctx.handle, L.fptr(s), len(s), L.fptr(d), len(d),
                                            L.fptr(cs), L.fptr(cd), L.iptr(ii), L.fptr(sd),
                                            int(max_iter), L.fptr(out), C.byref(cost),
                                            C.byref(its)), "rst_gicp_solve")
    else:
        raise TypeError("ComputeAlignment(src, dst, T) or "
                        "ComputeAlignment(src, dst, src_covs, dst_covs, dst_indices, seed, T)")
    if st != L.RST_OK:
        return float("inf")
    T[...] = L.cm_to_pose(out)
    return float(cost.value)


def ComputeNormals(cloud, tree: Target, num_neighbors: int = 16,
                   viewpoint=(0.0, 0.0, 0.0)) -> np.ndarray:
    """kNN-PCA normals of `tree`'s cloud, oriented toward `viewpoint`
    (the reference always follows ComputeNormals with OrientNormals:
    fpfh.cpp:247-248, rs_replay_app.cpp:386-387)."""
    tree.compute_normals(int(num_neighbors), viewpoint)
    return tree.normals()


def OrientNormals(cloud, viewpoint, normals: np.ndarray) -> None:
    """point_cloud_utils.cpp:206-216: flip n where (p - viewpoint).n > 0."""
    p = L.as_cloud(cloud)
    v = np.asarray(viewpoint, np.float32)
    ray = p - v
    dot = ray[:, 0] * normals[:, 0] + (ray[:, 1] * normals[:, 1] + ray[:, 2] * normals[:, 2])
    normals[dot > 0] *= -1.0
