"""Far-point certificate rule of the ICP search kernels (icp.hip: the fallback
keeps the two nearest and stores (q0, g = sqrt(d2_2nd) * 0.99999); kernel 1
accepts the stored neighbour p for a later query q without searching when
sqrt(d2(q, p)) * 1.00001 + |q - q0| * 1.00001 + 1e-30 < g).

CPU property test of that predicate in the kernel's float32 arithmetic
(d2 = (dx*dx + dy*dy) + dz*dz, each operation rounded, no contraction): on
every query the rule accepts, the brute-force exact nearest neighbour under
the reference's order ((d2, index), align_icp.cpp:112 through nanoflann) must
be p.  Queries are drawn around q0 at moves from far below to just above the
certificate's reach, on clouds with duplicate points and near-ties."""
import numpy as np

f32 = np.float32


def d2_ref(q, pts):
    d = (pts - q).astype(f32)
    return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]


def nearest(q, pts):
    d2 = d2_ref(q, pts)
    order = np.lexsort((np.arange(len(pts)), d2))
    return order[0], order[1], d2


def certified(q, p_xyz, q0, g):
    dp = (q - p_xyz).astype(f32)
    dq = (q - q0).astype(f32)
    dist_p = np.sqrt((dp[0] * dp[0] + dp[1] * dp[1]) + dp[2] * dp[2], dtype=f32)
    moved = np.sqrt((dq[0] * dq[0] + dq[1] * dq[1]) + dq[2] * dq[2], dtype=f32) * f32(1.00001)
    return dist_p * f32(1.00001) + moved + f32(1e-30) < g


def _cloud(rng, n, dup):
    pts = rng.uniform(-1, 1, (n, 3)).astype(f32)
    if dup:  # exact duplicates and points one float ulp apart
        k = n // 8
        pts[-k:] = pts[:k]
        pts[-2 * k:-k] = np.nextafter(pts[k:2 * k], f32(2))
    return pts


def test_certificate_rule_accepts_only_the_exact_nearest():
    rng = np.random.default_rng(3)
    accepted = 0
    for trial in range(40):
        pts = _cloud(rng, 400, dup=trial % 2 == 1)
        for _ in range(20):
            q0 = (rng.uniform(-1.2, 1.2, 3)).astype(f32)
            p, second, d2 = nearest(q0, pts)
            g = np.sqrt(d2[second], dtype=f32) * f32(0.99999)
            if not g > 0:
                continue  # a duplicate of the answer: no certificate
            for scale in (1e-4, 1e-2, 0.25, 0.5, 0.55, 1.0):
                for _ in range(4):
                    u = rng.normal(size=3)
                    q = (q0 + (u / np.linalg.norm(u)) * g * scale).astype(f32)
                    if certified(q, pts[p], q0, g):
                        accepted += 1
                        best, _, _ = nearest(q, pts)
                        assert best == p, (trial, scale)
    assert accepted > 1000  # the rule does fire on most small moves


def test_certificate_rule_rejects_ties():
    # q equidistant from two points: no certificate may hold
    pts = np.array([[0, 0, 0], [1, 0, 0], [0.5, 3, 0]], f32)
    q0 = np.array([0.1, 0, 0], f32)
    p, second, d2 = nearest(q0, pts)
    assert p == 0
    g = np.sqrt(d2[second], dtype=f32) * f32(0.99999)
    q_tie = np.array([0.5, 0, 0], f32)
    assert not certified(q_tie, pts[p], q0, g)
