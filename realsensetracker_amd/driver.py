"""Frame sources decoupled from the camera (rs_tracker/driver replacement).

    RandomSource(size, timestep, seed).GetCloud(prev_stamp) -> (cloud, stamp)
        data_source.hpp:22-41 (the reference's is unseeded setRandom())
    SyntheticScene(seed).render(T_wc, K) -> u16 depth image
        stands in for RealsenseSource / RsDriver (data_source_rs.cpp,
        rs_driver.cpp), which need a USB camera
    unproject(depth, K) -> (n, 3) float32 on the GPU
        rs2::pointcloud::calculate + ConvertPointCloud (data_source_rs.cpp:5-56)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .align import Context, get_context


def intrinsics(width: int = 640, height: int = 480, fx: float | None = None,
               fy: float | None = None, cx: float | None = None, cy: float | None = None,
               depth_scale: float = 0.001, min_depth: float = 0.3,
               max_depth: float = 5.0) -> L.Intrinsics:
    """RealSense-like pinhole (640x480 fx=fy~385; x2 at 720p)."""
    f = 385.0 * width / 640.0
    K = L.Intrinsics()
    K.fx = f if fx is None else fx
    K.fy = f if fy is None else fy
    K.cx = width / 2.0 if cx is None else cx
    K.cy = height / 2.0 if cy is None else cy
    K.width, K.height = width, height
    K.depth_scale, K.min_depth, K.max_depth = depth_scale, min_depth, max_depth
    return K


class SyntheticScene:
    """Seeded procedural room with spheres and boxes; ray-cast u16 depth."""

    def __init__(self, seed: int = 0):
        self._h = C.c_void_p()
        L.check(L.lib().rst_scene_create(seed, C.byref(self._h)), "rst_scene_create")

    def render(self, T_wc, K: L.Intrinsics, noise_seed: int = 0, noise_sigma: float = 0.001,
               invalid_frac: float = 0.03) -> np.ndarray:
        buf = L.pose_to_cm(T_wc)
        out = np.zeros((K.height, K.width), np.uint16)
        L.check(L.lib().rst_scene_render_depth(self._h, L.fptr(buf), C.byref(K), noise_seed,
                                               noise_sigma, invalid_frac, L.u16ptr(out)),
                "rst_scene_render_depth")
        return out

    def trajectory(self, frame: int) -> np.ndarray:
        buf = np.zeros(16, np.float32)
        L.check(L.lib().rst_scene_trajectory(self._h, frame, L.fptr(buf)), "trajectory")
        return L.cm_to_pose(buf)

    def __del__(self):
        try:
            if self._h:
                L.lib().rst_scene_destroy(self._h)
        except Exception:
            pass


class RandomSource:
    """data_source.hpp:22-41: uniform [-1,1]^3 clouds of `size` points."""

    def __init__(self, size: int = 128, timestep: float = 0.1, seed: int = 0):
        self.size, self.timestep, self.seed = size, timestep, seed
        self._k = 0

    def GetCloud(self, prev_stamp: float):
        out = np.zeros((self.size, 3), np.float32)
        L.check(L.lib().rst_random_cloud(self.seed * 1000003 + self._k, self.size,
                                         L.fptr(out)), "rst_random_cloud")
        self._k += 1
        return out, prev_stamp + self.timestep


def unproject(depth: np.ndarray, K: L.Intrinsics, keep_invalid: bool = False,
              ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or get_context()
    d = np.ascontiguousarray(depth, dtype=np.uint16)
    out = np.zeros((K.width * K.height, 3), np.float32)
    n = C.c_int64(0)
    L.check(L.lib().rst_unproject(ctx.handle, L.u16ptr(d), C.byref(K), int(keep_invalid),
                                  L.fptr(out), C.byref(n)), "rst_unproject")
    return out[: n.value].copy()


def se3_exp(rotvec, trans) -> np.ndarray:
    """4x4 from axis-angle (rad) and translation (m), float64 math."""
    w = np.asarray(rotvec, np.float64)
    th = float(np.linalg.norm(w))
    Kx = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        R = np.eye(3) + Kx
    else:
        R = np.eye(3) + np.sin(th) / th * Kx + (1 - np.cos(th)) / th**2 * Kx @ Kx
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = trans
    return T


def random_offset(rng: np.random.Generator, deg=(1.0, 3.0), cm=(1.0, 3.0)) -> np.ndarray:
    """Known SE(3) offset: |theta| in deg range, |t| in cm range."""
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    th = np.deg2rad(rng.uniform(*deg))
    tv = rng.normal(size=3)
    tv /= np.linalg.norm(tv)
    return se3_exp(ax * th, tv * rng.uniform(*cm) / 100.0)


def make_pair(scene: SyntheticScene, K: L.Intrinsics, seed: int, T_wa=None,
              noise_sigma: float = 0.001, invalid_frac: float = 0.03):
    """Two frames a, b at a known offset.  Returns (depth_a, depth_b, T_ab)
    where T_ab maps camera-b points into camera a (the pose AlignIcp3d(src=b,
    dst=a) should find)."""
    rng = np.random.default_rng(seed)
    T_wa = np.eye(4) if T_wa is None else np.asarray(T_wa, np.float64)
    D = random_offset(rng)
    T_wb = T_wa @ D
    da = scene.render(T_wa.astype(np.float32), K, 2 * seed + 1, noise_sigma, invalid_frac)
    db = scene.render(T_wb.astype(np.float32), K, 2 * seed + 2, noise_sigma, invalid_frac)
    return da, db, D
