"""Pixel-window rule of the ICP's frame-target searches (rst_wave_nn.hpp
pix_window / pix_tile_search / row_pix): a frame's point of level pixel
(a, b) lies on the ray of full-resolution pixel (a s, b s), so for a query q
with q.z > 2 r every target point within r of q projects into the window

    |u - u_q| <= |fx| r sqrt(q.x^2 + q.z^2) / (q.z (q.z - r)) / s  (* 1.001 + 0.02 px)

(likewise v), with r = max(the seed distance with margins, 1.5 level
pixels at q's depth).  CPU property test of that bound in the kernel's
float32 arithmetic on synthetic depth frames (levels 1 and 2, noise and
invalid pixels): every target point within r of the query lies in the
window, so the window's (d2, index) minimum is the exact nearest
neighbour under the reference's order (align_icp.cpp:112 through
nanoflann)."""
import numpy as np
import pytest

from oracle import oracle as O
from realsensetracker_amd import driver

f32 = np.float32
MAXH, MINPX = f32(6.0), f32(1.5)


def window(K4, s, wl, hl, q, d0):
    """pix_window, operation for operation in float32; None = not applicable."""
    fx, fy, cx, cy = (f32(v) for v in K4)
    qx, qy, qz = (f32(v) for v in q)
    if not (d0 < np.finfo(f32).max) or not qz > 0:
        return None
    afx, afy = abs(fx), abs(fy)
    rw = max(np.sqrt(f32(d0)) * f32(1.00001) + f32(4e-6), MINPX * f32(s) * qz / min(afx, afy))
    if not qz > f32(2.0) * rw:
        return None
    iz = f32(1.0) / qz
    uq = (fx * qx * iz + cx) / f32(s)
    vq = (fy * qy * iz + cy) / f32(s)
    k = rw / (qz * (qz - rw)) / f32(s)
    bx = afx * k * np.sqrt(qx * qx + qz * qz) * f32(1.001) + f32(0.02)
    by = afy * k * np.sqrt(qy * qy + qz * qz) * f32(1.001) + f32(0.02)
    if not (bx <= MAXH and by <= MAXH):
        return None
    a0, a1 = max(0, int(np.ceil(uq - bx))), min(wl - 1, int(np.floor(uq + bx)))
    b0, b1 = max(0, int(np.ceil(vq - by))), min(hl - 1, int(np.floor(vq + by)))
    if a0 > a1 or b0 > b1:
        return None
    return a0, a1, b0, b1, rw


def d2_ref(q, pts):
    d = (pts - np.asarray(q, f32)).astype(f32)
    return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]


@pytest.mark.parametrize("stride", [1, 2])
def test_pixel_window_holds_every_point_within_r(stride):
    K = driver.intrinsics(160, 120)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    da, _, _ = driver.make_pair(driver.SyntheticScene(2), K, seed=5)
    h, w = da.shape
    wl, hl = (w + stride - 1) // stride, (h + stride - 1) // stride
    grid = O.unproject(da, K4, keep_invalid=True, stride=stride).reshape(hl, wl, 3)
    valid = da[::stride, ::stride][:hl, :wl] != 0
    vb, va = np.nonzero(valid)
    pts = grid[vb, va]  # row-major valid pixels = the frame's original order
    rng = np.random.default_rng(stride)
    checked = 0
    for _ in range(1500):
        j = rng.integers(len(pts))
        scale = 10.0 ** rng.uniform(-3.5, -1.3)  # 0.3 mm .. 5 cm off the surface
        q = (pts[j] + rng.normal(0, scale, 3)).astype(f32)
        d2 = d2_ref(q, pts)
        # seed: some target point near the query (as the ICP's last neighbour)
        near = np.argsort(d2)[:50]
        seed = near[rng.integers(len(near))]
        win = window(K4, stride, wl, hl, q, d2[seed])
        if win is None:
            continue
        a0, a1, b0, b1, rw = win
        inside = (va >= a0) & (va <= a1) & (vb >= b0) & (vb <= b1)
        true_d = np.linalg.norm(pts.astype(np.float64) - q.astype(np.float64), axis=1)
        assert inside[true_d <= float(rw)].all()
        # the window's (d2, index) minimum is the exact nearest neighbour
        order = np.lexsort((np.arange(len(pts)), d2))
        best = order[0]
        assert inside[best]
        cand = np.nonzero(inside)[0]
        wb = cand[np.lexsort((cand, d2[cand]))[0]]
        assert wb == best
        checked += 1
    assert checked > 1000
