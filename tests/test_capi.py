"""CPU: the C-ABI library loads, exports exactly what include/rst_align.h
declares, and its host-only entry points behave (no GPU compute here)."""
from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

from realsensetracker_amd import _lib as L
from realsensetracker_amd import driver

ROOT = Path(__file__).resolve().parents[1]


def declared_functions() -> list[str]:
    src = (ROOT / "include" / "rst_align.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rst_[a-z0-9_]+)\s*\(", src)))


def declared_debug_functions() -> list[str]:
    src = (ROOT / "include" / "rst_debug.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rst_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) >= 35
    dbg = declared_debug_functions()
    assert "rst_debug_stream_copy" in dbg
    lib = C.CDLL(str(L.LIB_PATH))
    missing = [n for n in names + dbg if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(L.PROTOTYPES) == declared_functions()


def test_abi_version_and_status_strings():
    lib = L.lib()
    assert lib.rst_abi_version() == 1
    for s in (0, 1, -1, -2, -3, -4, -5, -6):
        assert lib.rst_status_string(s)


def test_default_opts_are_reference_constants():
    o = L.default_opts()
    assert o.max_iter == 128            # rs_align_app.cpp:303 / rs_replay_app.cpp:251
    assert o.mode == L.RST_P2POINT_REF
    assert o.mu0 == np.float32(1.0)     # align_icp.cpp:91
    assert o.anneal_every == 8          # align_icp.cpp:96
    assert o.anneal_div == np.float32(1.4)
    assert o.sum_mode == L.RST_SUM_REF  # the reference's sequential fp32 sums
    assert C.sizeof(L.IcpOpts) == 64    # layout unchanged: sum_mode took a reserved word


def test_library_is_the_only_hip_runtime():
    """_lib.lib() maps exactly one libamdhip64 (no torch import behind it)."""
    import sys
    L.lib()
    assert "torch" not in sys.modules or L.hip_runtimes_mapped()
    assert len(L.hip_runtimes_mapped()) <= 1


def test_no_device_fails_loudly():
    if L.device_count() > 0:
        pytest.skip("GPU present")
    h = C.c_void_p()
    assert L.lib().rst_ctx_create(0, C.byref(h)) == -4  # RST_E_NODEVICE
    from realsensetracker_amd import align as A
    with pytest.raises(L.RstError):
        A.Context(0)


def test_scene_render_deterministic_and_plausible():
    K = driver.intrinsics(64, 48)
    sc = driver.SyntheticScene(3)
    T = np.eye(4, dtype=np.float32)
    a = sc.render(T, K, noise_seed=5)
    b = driver.SyntheticScene(3).render(T, K, noise_seed=5)
    assert np.array_equal(a, b)
    valid = a > 0
    assert 0.9 < valid.mean() < 0.995          # ~3 % dropped
    z = a[valid] * 1e-3
    assert z.min() >= 0.3 and z.max() <= 5.0
    c = sc.render(T, K, noise_seed=6)
    assert not np.array_equal(a, c)


def test_trajectory_motion_per_frame():
    sc = driver.SyntheticScene(0)
    for f in range(0, 90, 7):
        A = sc.trajectory(f).astype(np.float64)
        B = sc.trajectory(f + 1).astype(np.float64)
        D = np.linalg.inv(A) @ B
        ang = np.arccos(np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1))
        assert np.degrees(ang) < 4 and np.linalg.norm(D[:3, 3]) < 0.04


def test_random_source():
    rs = driver.RandomSource(128, 0.1, seed=1)
    c1, t1 = rs.GetCloud(0.0)
    c2, t2 = rs.GetCloud(t1)
    assert c1.shape == (128, 3) and c1.dtype == np.float32
    assert np.all(np.abs(c1) <= 1) and not np.array_equal(c1, c2)
    assert t1 == pytest.approx(0.1) and t2 == pytest.approx(0.2)


def test_pose_layout_roundtrip():
    T = np.arange(16, dtype=np.float32).reshape(4, 4)
    b = L.pose_to_cm(T)
    assert b[1] == T[1, 0] and b[4] == T[0, 1]   # column-major (Isometry3f::matrix())
    assert np.array_equal(L.cm_to_pose(b), T)
