"""Frame records of the replay path: the raw format
of include/rs_tracker/driver/cloud_record.hpp (the reference's protobuf
PointCloud schema is not vendored).  One frame per file:

    "RSTC" | u32 version=1 | u64 n | f64 stamp | u32 flags=0 | u32 0 | f32 xyz[n][3]
"""
from __future__ import annotations

import struct
from pathlib import Path

import numpy as np

_HDR = struct.Struct("<4sIQdII")
MAGIC = b"RSTC"


def write_record(path, cloud, stamp: float = 0.0) -> None:
    a = np.ascontiguousarray(np.asarray(cloud, np.float32).reshape(-1, 3))
    with open(path, "wb") as f:
        f.write(_HDR.pack(MAGIC, 1, a.shape[0], float(stamp), 0, 0))
        f.write(a.tobytes())


def read_record(path) -> tuple[np.ndarray, float]:
    with open(path, "rb") as f:
        magic, ver, n, stamp, _, _ = _HDR.unpack(f.read(_HDR.size))
        if magic != MAGIC or ver != 1:
            raise ValueError(f"{path}: not an RSTC v1 record")
        data = np.frombuffer(f.read(12 * n), np.float32)
        if data.size != 3 * n:
            raise ValueError(f"{path}: truncated record")
    return data.reshape(n, 3).copy(), stamp


def glob_records(directory) -> list[Path]:
    """The replay order: file names sorted (rs_replay_app.cpp's Glob)."""
    return sorted(Path(directory).glob("*.rstc"))
