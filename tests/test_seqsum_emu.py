"""Host emulation of the parallel sequential sums (seqsum.hip's kernels, one
workgroup after another, the same arithmetic header) against numpy's
sequential float32 accumulate -- the reference's `+=` loops
(align_icp.cpp:113,120; point_cloud_utils.cpp:94-96) -- bit for bit, under
ASan/UBSan: the map logic and every table bound, on the CPU."""
import numpy as np
import pytest

from seqsum_cases import cases
from seqsum_emu import emulate

CASES = cases()


def want(x):
    x = np.concatenate([np.zeros((1, 4), np.float32), np.asarray(x, np.float32)])
    with np.errstate(all="ignore"):
        return np.add.accumulate(x, axis=0, dtype=np.float32)[-1].view(np.uint32)


def same(got, w):
    g, w = np.asarray(got, np.uint32), np.asarray(w, np.uint32)
    gn, wn = np.isnan(g.view(np.float32)), np.isnan(w.view(np.float32))
    return np.array_equal(gn, wn) and np.array_equal(g[~gn], w[~wn])


@pytest.mark.parametrize("name", sorted(CASES))
def test_emulated_maps_bitexact(name):
    got, _ = emulate(CASES[name], sanitize=True)
    assert same(got, want(CASES[name])), name


def test_emulated_frame_chain_takes_superblock_jumps():
    """A 640x480-sized smooth chain: almost every superblock is one verified jump."""
    rng = np.random.default_rng(3)
    n = 307200
    u = np.tile(np.arange(640), 480)
    x = np.stack([(u - 320) / 385.0 * 2.0, np.full(n, 1.0), 2.0 + rng.normal(size=n) * 0.01,
                  rng.random(n)], 1).astype(np.float32)
    got, st = emulate(x)
    assert same(got, want(x))
    assert (st[:, 1] >= st[:, 0] - 2).all(), st
