"""Shared test setup.  `-m gpu` tests need an MI355X and the built HIP
library; `-m "not gpu"` tests run on CPU (oracle, host logic, C-ABI load)."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU and the built HIP library")


def _has_gpu() -> bool:
    try:
        from realsensetracker_amd import _lib as L
        return L.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_golden(name: str) -> dict:
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


GOLDEN_NAMES = sorted(p.stem for p in GOLDEN.glob("*.npz"))
PAIR_NAMES = [n for n in GOLDEN_NAMES if n.startswith("pair_")]


@pytest.fixture(scope="session")
def ctx():
    from realsensetracker_amd import align as A
    return A.get_context(0)
