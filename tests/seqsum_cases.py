"""Float4 streams for the sequential-sum tests (shared by the GPU tests and
the host emulation): mixed magnitudes at block / tile edges, exact ties,
zero crossings, alternating signs, overflow, subnormals, NaN / inf, zeros."""
import numpy as np


def cases():
    rng = np.random.default_rng(7)
    out = {}
    for n in (1, 2, 63, 64, 65, 4095, 4096, 4097, 262144 + 17):
        x = (rng.normal(size=(n, 4)) * 10 ** rng.uniform(-3, 2, size=(n, 4))).astype(np.float32)
        x[:, 3] = np.abs(x[:, 3])
        out[f"mixed_{n}"] = x
    n = 200_000
    # exact ties everywhere: small integers times powers of two
    out["ties"] = (rng.integers(-64, 64, size=(n, 4)) *
                   2.0 ** rng.integers(-12, 3, size=(n, 4))).astype(np.float32)
    # a sum that oscillates through zero (many binade changes)
    t = np.arange(n)
    osc = np.sin(t * 2 * np.pi / 640.0) + 1e-3 * rng.normal(size=n)
    out["zero_crossings"] = np.stack([osc, -osc, osc * 1e-3, np.abs(osc)], 1).astype(np.float32)
    # alternating +-, a constant (every add rounds the same way), growth to 2^24 and past it
    out["alternating"] = np.stack([(-1.0) ** t, (-1.0) ** t * 3.3, np.full(n, 0.1),
                                   np.full(n, 1.0)], 1).astype(np.float32)
    big = np.full((n, 4), 1e30, np.float32)
    big[:, 1] = 3e38  # overflows to +inf
    big[:, 2] = rng.normal(size=n) * 1e37
    out["huge"] = big
    tiny = (rng.normal(size=(n, 4)) * 1e-39).astype(np.float32)  # subnormals
    tiny[::1000, 1] = 1.0
    out["subnormal"] = tiny
    nf = (rng.normal(size=(n, 4))).astype(np.float32)
    nf[1000, 0] = np.nan
    nf[5000, 1] = np.inf
    nf[7000, 2] = np.inf
    nf[9000, 2] = -np.inf
    nf[150000, 3] = np.inf
    out["nonfinite"] = nf
    # the reference callers' sizes (5 cm voxel clouds, ~15k points)
    for name in ("ties", "zero_crossings", "alternating", "huge", "subnormal"):
        out[f"{name}_small"] = out[name][:15239].copy()
    nfs = out["nonfinite"][:16384].copy()
    nfs[12000, 3] = np.nan
    out["nonfinite_small"] = nfs
    for n in (16384, 16385):
        out[f"mixed_{n}"] = (rng.normal(size=(n, 4)) * 10 ** rng.uniform(-3, 2, size=(n, 4))).astype(np.float32)
    out["zeros"] = np.zeros((5000, 4), np.float32)
    neg0 = np.full((100, 4), -0.0, np.float32)
    out["neg_zeros"] = neg0
    return out


