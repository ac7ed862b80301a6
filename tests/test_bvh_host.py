"""CPU check of the GPU's exact-NN searches (rst_bvh.hpp is
__host__ __device__): tests/cpp/bvh_selftest.cpp builds the index on the CPU
and compares top-down, bottom-up (warm) and k-NN searches with brute force
on random, lattice (ties/duplicates), surface-like and non-finite clouds."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "cpp" / "bvh_selftest.cpp"
CSRC = ROOT / "realsensetracker_amd" / "csrc"


@pytest.fixture(scope="module")
def selftest(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("bvh") / "bvh_selftest"
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-x", "hip",
                    "--offload-arch=gfx950", f"-I{CSRC}", str(SRC), "-o", str(out)],
                   check=True, capture_output=True)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bvh_searches_exact_on_cpu(selftest, seed):
    r = subprocess.run([str(selftest), str(seed)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
