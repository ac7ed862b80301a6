"""SURVEY.md §5 (sanitizers on host code): the CPU oracle built with
-fsanitize=address,undefined (oracle/Makefile `asan`) and driven over every
entry point of rst_oracle.h by oracle/asan_main.c on a seeded synthetic
frame, including NaN/inf clouds and 0-3 point edge sizes.  Any ASan or
UBSan report aborts the binary (-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ORACLE = Path(__file__).resolve().parents[1] / "oracle"


@pytest.mark.skipif(shutil.which("make") is None or shutil.which("gcc") is None,
                    reason="no host toolchain")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", str(ORACLE), "asan"], check=True, timeout=300)
    # (verify_asan_link_order=0: the environment may preload its own library)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="2")
    p = subprocess.run([str(ORACLE / "_asan" / "rst_oracle_asan")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "sanitizer run ok" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
