"""ctypes binding of the C ABI in include/rst_align.h.

The product path has exactly one implementation: the HIP library
``realsensetracker_amd/lib/librst_align.so``.  If it is missing or cannot be
loaded this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ.get("RST_LIB")  # (an empty value: the default)
                or Path(__file__).resolve().parent / "lib" / "librst_align.so")

RST_OK, RST_FALSE = 0, 1
RST_E_ARG, RST_E_HIP, RST_E_NOMEM, RST_E_NODEVICE, RST_E_COMM, RST_E_STATE = -1, -2, -3, -4, -5, -6
RST_P2POINT_REF, RST_P2PLANE = 0, 1
RST_SUM_REF, RST_SUM_FP64 = 0, 1  # rst_sum_mode: reference fp32 sequential sums / fp64 sums
COMM_ID_BYTES = 128

c_float_p = C.POINTER(C.c_float)
c_int32_p = C.POINTER(C.c_int32)
c_int64_p = C.POINTER(C.c_int64)
c_u16_p = C.POINTER(C.c_uint16)


class IcpOpts(C.Structure):
    _fields_ = [("max_iter", C.c_int32), ("mode", C.c_int32), ("mu0", C.c_float),
                ("anneal_every", C.c_int32), ("anneal_div", C.c_float),
                ("p2plane_eps", C.c_float), ("p2plane_mu", C.c_float),
                ("p2plane_max_dist", C.c_float), ("sum_mode", C.c_int32),
                ("n_total", C.c_int32), ("reserved", C.c_int32 * 6)]


class Intrinsics(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("width", C.c_int32), ("height", C.c_int32), ("depth_scale", C.c_float),
                ("min_depth", C.c_float), ("max_depth", C.c_float)]


_P = C.c_void_p
# name -> (restype, argtypes); mirrors include/rst_align.h one to one
PROTOTYPES = {
    "rst_abi_version": (C.c_int, []),
    "rst_status_string": (C.c_char_p, [C.c_int]),
    "rst_icp_opts_default": (None, [C.POINTER(IcpOpts)]),
    "rst_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rst_ctx_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "rst_dev_alloc": (C.c_int, [_P, C.c_int64, C.POINTER(_P)]),
    "rst_dev_free": (C.c_int, [_P, _P]),
    "rst_dev_upload": (C.c_int, [_P, _P, _P, C.c_int64]),
    "rst_dev_download": (C.c_int, [_P, _P, _P, C.c_int64]),
    "rst_ctx_destroy": (C.c_int, [_P]),
    "rst_ctx_set_stream": (C.c_int, [_P, _P]),
    "rst_ctx_synchronize": (C.c_int, [_P]),
    "rst_ctx_last_kernel_time": (C.c_int, [_P, c_float_p, c_int32_p]),
    "rst_ctx_last_iteration_times": (C.c_int, [_P, c_float_p, c_int32_p]),
    "rst_ctx_last_iterations": (C.c_int, [_P, c_int32_p]),
    "rst_ctx_enable_kernel_timing": (C.c_int, [_P, C.c_int]),
    "rst_target_build": (C.c_int, [_P, c_float_p, C.c_int64, C.POINTER(_P)]),
    "rst_target_build_device": (C.c_int, [_P, _P, C.c_int64, C.POINTER(_P)]),
    "rst_target_free": (C.c_int, [_P]),
    "rst_target_size": (C.c_int64, [_P]),
    "rst_target_compute_normals": (C.c_int, [_P, _P, C.c_int, c_float_p]),
    "rst_target_compute_grid_normals": (C.c_int, [_P, _P, C.c_int, c_float_p]),
    "rst_target_get_normals": (C.c_int, [_P, _P, c_float_p]),
    "rst_target_query_nn": (C.c_int, [_P, _P, c_float_p, C.c_int64, c_int32_p, c_float_p]),
    "rst_target_query_nn_device": (C.c_int, [_P, _P, _P, C.c_int64, _P, _P]),
    "rst_target_query_nn_warm": (C.c_int, [_P, _P, c_float_p, C.c_int64, c_int32_p, c_int32_p,
                                           c_float_p]),
    "rst_target_query_knn": (C.c_int, [_P, _P, c_float_p, C.c_int64, C.c_int, c_int32_p,
                                       c_float_p]),
    "rst_icp_align": (C.c_int, [_P, c_float_p, C.c_int64, _P, C.POINTER(IcpOpts), c_float_p,
                                c_float_p]),
    "rst_icp_align_clouds": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p, C.c_int64,
                                       C.POINTER(IcpOpts), c_float_p, c_float_p]),
    "rst_icp_align_device": (C.c_int, [_P, _P, C.c_int64, _P, C.POINTER(IcpOpts), c_float_p,
                                       c_float_p]),
    "rst_icp_align_prepared": (C.c_int, [_P, _P, _P, C.POINTER(IcpOpts), c_float_p, c_float_p,
                                         c_int32_p]),
    "rst_solve_kabsch": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p, C.c_int64, c_int32_p,
                                   c_float_p, C.c_int64, c_float_p]),
    "rst_icp_align_prepared_async": (C.c_int, [_P, _P, _P, C.POINTER(IcpOpts), c_float_p]),
    "rst_icp_align_wait": (C.c_int, [_P, c_float_p, c_float_p, c_int32_p]),
    "rst_icp_align_batch_async": (C.c_int, [_P, C.c_int32, C.POINTER(_P), C.POINTER(_P),
                                            C.POINTER(IcpOpts), c_float_p]),
    "rst_icp_align_batch_wait": (C.c_int, [_P, c_float_p, c_float_p, c_int32_p, c_int32_p]),
    "rst_ctx_enable_graphs": (C.c_int, [_P, C.c_int]),
    "rst_icp_align_pyramid_async": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.c_int,
                                              c_int32_p, C.POINTER(IcpOpts), c_float_p]),
    "rst_compute_centroid": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p]),
    "rst_kabsch_solve": (C.c_int, [_P, C.POINTER(C.c_double), c_float_p, c_float_p, c_float_p]),
    "rst_unproject": (C.c_int, [_P, c_u16_p, C.POINTER(Intrinsics), C.c_int, c_float_p,
                                c_int64_p]),
    "rst_unproject_device": (C.c_int, [_P, _P, C.POINTER(Intrinsics), C.c_int, _P, c_int64_p]),
    "rst_unproject_strided_device": (C.c_int, [_P, _P, C.POINTER(Intrinsics), C.c_int, C.c_int,
                                               _P, c_int64_p]),
    "rst_remove_nans": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p, c_int64_p]),
    "rst_remove_nans_device": (C.c_int, [_P, _P, C.c_int64, _P, c_int64_p]),
    "rst_downsample_voxel": (C.c_int, [_P, c_float_p, C.c_int64, C.c_float, c_float_p,
                                       c_int64_p]),
    "rst_downsample_voxel_device": (C.c_int, [_P, _P, C.c_int64, C.c_float, _P, c_int64_p]),
    "rst_compute_fpfh": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p, C.c_int, C.c_float,
                                   c_float_p]),
    "rst_compute_matches": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p, C.c_int64, C.c_int,
                                      c_int32_p, c_float_p]),
    "rst_accum_create": (C.c_int, [_P, C.c_float, C.POINTER(_P)]),
    "rst_accum_destroy": (C.c_int, [_P]),
    "rst_accum_add": (C.c_int, [_P, c_float_p, c_float_p, C.c_int64]),
    "rst_accum_add_device": (C.c_int, [_P, c_float_p, _P, C.c_int64]),
    "rst_accum_size": (C.c_int, [_P, c_int64_p]),
    "rst_accum_extract": (C.c_int, [_P, c_float_p, c_int64_p]),
    "rst_compute_covariances": (C.c_int, [_P, _P, C.c_int, c_float_p]),
    "rst_gicp_solve": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p, C.c_int64, c_float_p,
                                 c_float_p, c_int32_p, c_float_p, C.c_int, c_float_p,
                                 C.POINTER(C.c_double), c_int32_p]),
    "rst_gicp_align": (C.c_int, [_P, c_float_p, C.c_int64, c_float_p, C.c_int64, C.c_int,
                                 C.c_int, c_float_p, C.POINTER(C.c_double)]),
    "rst_frame_prepare_device": (C.c_int, [_P, _P, C.POINTER(Intrinsics), C.c_int,
                                           C.POINTER(_P)]),
    "rst_frame_prepare_pyramid_device": (C.c_int, [_P, _P, C.POINTER(Intrinsics), C.c_int,
                                                   C.c_int, C.POINTER(_P)]),
    "rst_scene_create": (C.c_int, [C.c_uint64, C.POINTER(_P)]),
    "rst_scene_destroy": (C.c_int, [_P]),
    "rst_scene_render_depth": (C.c_int, [_P, c_float_p, C.POINTER(Intrinsics), C.c_uint64,
                                         C.c_float, C.c_float, c_u16_p]),
    "rst_scene_trajectory": (C.c_int, [_P, C.c_int32, c_float_p]),
    "rst_random_cloud": (C.c_int, [C.c_uint64, C.c_int64, c_float_p]),
    "rst_comm_get_unique_id": (C.c_int, [C.c_char_p]),
    "rst_comm_create": (C.c_int, [_P, C.c_char_p, C.c_int, C.c_int, C.POINTER(_P)]),
    "rst_comm_destroy": (C.c_int, [_P]),
    "rst_icp_align_sharded_device": (C.c_int, [_P, _P, _P, C.c_int64, _P, C.POINTER(IcpOpts),
                                               c_float_p, c_float_p]),
    "rst_icp_align_sharded_prepared": (C.c_int, [_P, _P, _P, _P, C.POINTER(IcpOpts),
                                                 c_float_p, c_float_p]),
}

_lib = None


def hip_runtimes_mapped() -> list[str]:
    """Distinct libamdhip64 files mapped into this process (from
    /proc/self/maps).  Two means two HIP runtimes -- e.g. torch's bundled
    copy and /opt/rocm's -- which tear each other down at exit."""
    seen = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and "libamdhip64" in parts[-1]:
                    path = os.path.realpath(parts[-1])
                    if path not in seen:
                        seen.append(path)
    except OSError:
        pass
    return seen


def lib() -> C.CDLL:
    """Load librst_align.so (raises if it is absent: no fallback path).

    The library binds whichever HIP runtime the process already has mapped
    (the dynamic linker resolves its libamdhip64 soname to a loaded copy),
    else /opt/rocm's.  Loading it into a process that ends up with two
    runtimes mapped is refused."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(
                f"realsensetracker_amd: HIP library not built ({LIB_PATH}); run "
                "`python -m realsensetracker_amd.build` (or __graft_entry__.build())")
        # kernel arguments in device memory (the library's load-time default
        # too; here for a runtime that initialises before the library loads)
        if os.environ.get("RST_NO_ENV_DEFAULTS", "0") in ("", "0"):
            os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
        L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        rts = hip_runtimes_mapped()
        if len(rts) > 1:
            raise ImportError("realsensetracker_amd: two HIP runtimes mapped in this process "
                              f"({', '.join(rts)}); load the library before or without a "
                              "second runtime (e.g. torch's)")
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class RstError(RuntimeError):
    def __init__(self, status: int, what: str):
        msg = lib().rst_status_string(status)
        super().__init__(f"{what}: status {status} ({msg.decode() if msg else '?'})")
        self.status = status


def check(status: int, what: str) -> int:
    """Raise on negative status; return 0 (ok) / 1 (reference false)."""
    if status < 0:
        raise RstError(status, what)
    return status


def fptr(a: np.ndarray):
    return a.ctypes.data_as(c_float_p)


def iptr(a: np.ndarray):
    return a.ctypes.data_as(c_int32_p)


def u16ptr(a: np.ndarray):
    return a.ctypes.data_as(c_u16_p)


def as_cloud(x) -> np.ndarray:
    """Cloud3f <-> (n, 3) float32 C-contiguous (same bytes as Eigen 3xN col-major)."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    if a.ndim != 2 or a.shape[1] != 3:
        raise ValueError(f"cloud must be (n, 3), got {a.shape}")
    return a


def pose_to_cm(T) -> np.ndarray:
    """4x4 (math orientation) -> 16 float32 column-major (Isometry3f::matrix())."""
    T = np.asarray(T, dtype=np.float32).reshape(4, 4)
    return np.ascontiguousarray(T.T).reshape(16).copy()


def cm_to_pose(b) -> np.ndarray:
    return np.asarray(b, dtype=np.float32).reshape(4, 4).T.copy()


def default_opts(**kw) -> IcpOpts:
    o = IcpOpts()
    lib().rst_icp_opts_default(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def device_count() -> int:
    c = C.c_int(0)
    lib().rst_device_count(C.byref(c))
    return c.value
