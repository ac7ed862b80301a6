"""Build the MI355X library (HIP for gfx950) in-tree.

    python -m realsensetracker_amd.build           # library + app
    python -m realsensetracker_amd.build --lib     # library only

Outputs (git-ignored, shipped to the GPU box by gpurun):
    realsensetracker_amd/lib/librst_align.so   C-ABI of include/rst_align.h
    realsensetracker_amd/lib/rs_replay_app     host C++ replay app
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
OBJDIR = ROOT / "build" / "obj"
INCLUDE = ROOT / "include"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("RST_OFFLOAD_ARCH", "gfx950")

SOURCES = ["build.hip", "query.hip", "icp.hip", "seqsum.hip", "capi.hip", "unproject.hip", "voxel.hip", "gicp.hip", "fpfh.hip", "comm.hip", "synth.cpp"]
LIB_NAME = "librst_align.so"

# -ffp-contract=off: reference-exact rounding of the transform / distance /
# weight arithmetic (DESIGN.md "Numerics").
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
          "-Wall", "-Wno-unused-function", "-Wno-unused-result", f"-I{INCLUDE}", f"-I{CSRC}"]
# tuning experiments: RST_DEFINES="-DNAME=V ..." builds a variant library
# (python -m realsensetracker_amd.build --lib --out lib/variants/x.so; load
# it with RST_LIB=...)
CFLAGS += os.environ.get("RST_DEFINES", "").split()


def _hipcc() -> str:
    h = ROCM / "bin" / "hipcc"
    return str(h) if h.exists() else "hipcc"


def _stamp(src: Path) -> str:
    h = hashlib.sha1()
    # every header can reach every source: hash them all
    for p in [src] + sorted(CSRC.glob("*.hpp")) + sorted(INCLUDE.glob("*.h")):
        h.update(p.read_bytes())
    h.update(" ".join(CFLAGS).encode())
    return h.hexdigest()[:16]


def _compile(src: str) -> Path:
    s = CSRC / src
    obj = OBJDIR / (s.stem + "." + _stamp(s) + ".o")
    if obj.exists():
        return obj
    cmd = [_hipcc(), *CFLAGS, "-c", str(s), "-o", str(obj)]
    if src.endswith(".cpp"):
        cmd.insert(1, "-x")
        cmd.insert(2, "hip")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build_library(jobs: int = 8, out: Path | None = None) -> Path:
    OBJDIR.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(SOURCES)))) as ex:
        objs = list(ex.map(_compile, SOURCES))
    out = Path(out) if out else LIBDIR / LIB_NAME
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.with_name(out.name + ".tmp")
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp),
           *map(str, objs), f"-L{ROCM / 'lib'}", "-lrccl", f"-Wl,-rpath,{ROCM / 'lib'}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    if out == LIBDIR / LIB_NAME:
        (LIBDIR / "BUILD_INFO.json").write_text(json.dumps({"source_hash": source_hash()}) + "\n")
    return out


def source_hash() -> str:
    """Hash of every kernel / C-ABI source and the flags: identifies the
    code a measurement (PMC traffic, profiles) was taken on, on the GPU box
    too (no .git there)."""
    h = hashlib.sha1()
    for p in sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.hpp")) + sorted(CSRC.glob("*.cpp")) + \
            sorted(INCLUDE.glob("*.h")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(CFLAGS).encode())
    return h.hexdigest()[:16]


def build_app() -> Path:
    """Host C++ replay app over the C-ABI (rs_replay_app.cpp's loop)."""
    src = CSRC / "app" / "rs_replay_app.cpp"
    out = LIBDIR / "rs_replay_app"
    if not src.exists():
        return out
    cmd = ["g++", "-O2", "-std=c++17", f"-I{INCLUDE}", str(src), "-o", str(out),
           f"-L{LIBDIR}", "-lrst_align", "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"app build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="store_true", help="library only")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("--out", default=None, help="library path (variant builds)")
    a = ap.parse_args(argv)
    if a.clean and OBJDIR.exists():
        shutil.rmtree(OBJDIR)
    p = build_library(a.j, PKG / a.out if a.out else None)
    print(p)
    if not a.lib:
        print(build_app())
    return 0


if __name__ == "__main__":
    sys.exit(main())
