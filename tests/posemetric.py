"""Pose comparison used by the tests and bench (test/bench infrastructure)."""
from __future__ import annotations

import numpy as np


def pose_err(A, B):
    """(rotation angle in rad, translation distance in m) between two 4x4
    poses.  The angle is atan2(|skew(A B^T)|, (tr(A B^T) - 1) / 2), which stays
    accurate near zero (arccos of the trace alone reads ~1e-4 rad of noise
    for identical float32 rotations)."""
    A = np.asarray(A, np.float64)
    B = np.asarray(B, np.float64)
    dR = A[:3, :3] @ B[:3, :3].T
    w = 0.5 * np.array([dR[2, 1] - dR[1, 2], dR[0, 2] - dR[2, 0], dR[1, 0] - dR[0, 1]])
    ang = float(np.arctan2(np.linalg.norm(w), 0.5 * (np.trace(dR) - 1.0)))
    return ang, float(np.linalg.norm(A[:3, 3] - B[:3, 3]))
