"""Seeded clouds for the RemoveNans / DownsampleVoxel parity tests
(point_cloud_utils.cpp:34-68, 163-174): shared by the oracle (CPU) and the
GPU tests.  The reference has no tests of its own for these functions, so
the oracle is pinned against tests/np_restate.py (parity unpinned against
the reference binary, which cannot be built here)."""
from __future__ import annotations

import numpy as np

VOXEL = 0.05  # rs_replay_app.cpp:246-247, rs_align_app.cpp default


def frame_cloud(name: str = "pair_160x120_s2") -> np.ndarray:
    """An unprojected synthetic depth frame (structured, dense surfaces):
    the committed golden pair's source cloud."""
    from conftest import load_golden
    return load_golden(name)["src"]


def cases() -> dict[str, tuple[np.ndarray, float]]:
    rng = np.random.default_rng(7)
    out: dict[str, tuple[np.ndarray, float]] = {}
    out["empty"] = (np.zeros((0, 3), np.float32), VOXEL)
    out["one"] = (np.array([[0.1, -0.2, 0.3]], np.float32), VOXEL)
    u = rng.uniform(-2, 2, (5000, 3)).astype(np.float32)
    out["uniform_5000"] = (u, VOXEL)
    out["uniform_coarse"] = (u, 0.5)
    # every point on a voxel boundary (k * v), and just below it
    g = (rng.integers(-40, 40, (3000, 3)) * np.float32(VOXEL)).astype(np.float32)
    edge = np.concatenate([g, np.nextafter(g, np.float32(-np.inf))])
    out["voxel_edges"] = (edge[rng.permutation(len(edge))], VOXEL)
    # duplicates, NaN / inf rows, out-of-int-range coordinates
    d = rng.uniform(-1, 1, (4000, 3)).astype(np.float32)
    d[rng.integers(0, 4000, 300)] = d[rng.integers(0, 4000, 300)]
    d[rng.integers(0, 4000, 200), rng.integers(0, 3, 200)] = np.nan
    d[rng.integers(0, 4000, 50), rng.integers(0, 3, 50)] = np.inf
    d[rng.integers(0, 4000, 50), rng.integers(0, 3, 50)] = -np.inf
    d[rng.integers(0, 4000, 20), rng.integers(0, 3, 20)] = 3e30
    out["nonfinite_4000"] = (d, VOXEL)
    out["all_nan"] = (np.full((100, 3), np.nan, np.float32), VOXEL)
    return out
