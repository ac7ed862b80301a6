"""Build and run the host emulation of seqsum.hip (tests/cpp/seqsum_emu.cpp;
test infrastructure: it shares the kernels' arithmetic header and checks
the map logic and every table bound on the CPU)."""
import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "cpp" / "seqsum_emu.cpp"
HDR = ROOT / "realsensetracker_amd" / "csrc" / "rst_seqsum.hpp"
_BIN = None


def binary(sanitize: bool = False) -> Path:
    global _BIN
    if _BIN is not None:
        return _BIN
    out = Path(tempfile.gettempdir()) / f"rst_seqsum_emu_{os.getpid()}{'_asan' if sanitize else ''}"
    cmd = ["g++", "-O2", "-std=c++17", f"-I{HDR.parent}", str(SRC), "-o", str(out)]
    if sanitize:
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-g"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    _BIN = out
    return out


def emulate(x, sanitize=False, p0=None, s0=None):
    """(sums as uint32 bits [4], walk stats [4][10]) of a float4 stream.
    p0 (4 fp64) / s0 (4 float32): the stream is a stretch of a longer chain
    -- the fp64 prefix before it (the guesses' offset) and the chain's value
    where it starts (the walk's start), as the sharded loop's relay runs it."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1, 4)
    env = dict(os.environ)
    if p0 is not None:
        env["EMU_P0"] = ",".join(repr(float(v)) for v in p0)
    if s0 is not None:
        env["EMU_S0"] = ",".join("%08x" % int(v) for v in np.asarray(s0, np.float32).view(np.uint32))
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "in.f32"
        x.tofile(f)
        r = subprocess.run([str(binary(sanitize)), str(f), str(len(x)), "4"], capture_output=True,
                           text=True, env=env)
    if r.returncode != 0:
        raise RuntimeError(f"emulation failed: {r.stdout[-500:]} {r.stderr[-2000:]}")
    rows = [ln.split() for ln in r.stdout.splitlines() if ln.strip()]
    return (np.array([int(t[0], 16) for t in rows], np.uint32),
            np.array([[int(v) for v in t[1:]] for t in rows], np.int64))


def emulate_tables(x, c):
    """the front kernel's tables of chain c: bs, gs, ks, inc"""
    x = np.ascontiguousarray(x, np.float32).reshape(-1, 4)
    n = len(x)
    nb = (n + 15) // 16
    ng = (nb + 15) // 16
    nk = (ng + 15) // 16
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "in.f32"
        x.tofile(f)
        env = dict(os.environ, EMU_DUMP=str(Path(d) / "dump"))
        subprocess.run([str(binary()), str(f), str(n), "4"], check=True, capture_output=True, env=env)
        raw = (Path(d) / f"dump.{c}").read_bytes()
    ints = np.frombuffer(raw, np.int32, count=(nb + 1) + (ng + 1) + (nk + 1))
    bs, gs, ks = ints[:nb + 1], ints[nb + 1:nb + 1 + ng + 1], ints[nb + ng + 2:]
    inc = np.frombuffer(raw, np.float64, offset=4 * len(ints), count=nb)
    return bs, gs, ks, inc
