"""Process-group plumbing of one job (one process per GPU), without torch.

The HIP library must be the only HIP runtime in its process (``_lib.lib``
refuses a second one), so the multi-GPU bench and the sharded align do not
import torch for their host-side coordination.  What they need is small and
lives here:

* ``rank_envs`` / ``launch``: ``bench.py --gpus N`` run without a launcher
  spawns N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE /
  MASTER_ADDR / MASTER_PORT, the torch.distributed.run convention, so the
  same script also runs under ``python -m torch.distributed.run``);
* ``Rendezvous``: barrier, all-reduce (sum / max) of a few float64 values
  and a byte broadcast (the RCCL unique id) over TCP, rank 0 serving at
  MASTER_ADDR:MASTER_PORT.  Only timing and setup go through it; the data
  path's exchange is RCCL inside librst_align.so.
"""
from __future__ import annotations

import os
import socket
import struct
import signal
import subprocess
import sys
import threading
import time

import numpy as np

_HDR = struct.Struct("<q")


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def rank_envs(nproc: int, port: int, base: dict | None = None,
              addr: str = "127.0.0.1") -> list[dict]:
    """The environment of each of nproc local ranks (rank r on GPU r)."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(nproc):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc),
                 LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR=addr, MASTER_PORT=str(port))
        out.append(e)
    return out


def launch(nproc: int, argv: list[str], script: str, grace: float = 10.0,
           poll: float = 0.05, timeout: float | None = None) -> int:
    """Run `script argv` as nproc rank processes; the job's exit status is
    the first failing rank's (0 when all succeed).  Called before anything
    touches the GPU.

    All ranks are polled together: when one exits non-zero the others are
    sent SIGTERM (a rank blocked in a collective would otherwise wait for
    the dead peer until its own timeout), and whatever is still running
    `grace` seconds later is killed.  `timeout` (seconds, None = none)
    bounds the whole job the same way; the status is then 124."""
    envs = rank_envs(nproc, free_port())
    procs = [subprocess.Popen([sys.executable, script, *argv], env=e) for e in envs]
    status = 0
    t0 = time.monotonic()
    # a SIGTERM to the launcher stops the ranks too (no orphans); the
    # handler raises, and the except clause below reaps them
    prev_term = None
    if threading.current_thread() is threading.main_thread():
        def _on_term(signum, frame):
            raise SystemExit(128 + signum)
        prev_term = signal.signal(signal.SIGTERM, _on_term)
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c is not None and c != 0]
            if bad:
                # a rank killed by signal N reports -N: the shell's 128 + N
                status = 128 - bad[0] if bad[0] < 0 else bad[0]
                break
            if all(c is not None for c in codes):
                return 0
            if timeout is not None and time.monotonic() - t0 > timeout:
                status = 124
                break
            time.sleep(poll)
    except BaseException:
        _stop(procs, grace)
        raise
    finally:
        if prev_term is not None:
            signal.signal(signal.SIGTERM, prev_term)
    _stop(procs, grace)
    return status


def _stop(procs: list[subprocess.Popen], grace: float) -> None:
    """SIGTERM every rank still running, SIGKILL after `grace` seconds, and
    reap them all."""
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def world_from_env() -> tuple[int, int, int]:
    """(world, rank, local_rank) from the launcher's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _send(s: socket.socket, data: bytes) -> None:
    s.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(s: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed")
        buf += chunk
    return bytes(buf)


def _recv(s: socket.socket) -> bytes:
    (n,) = _HDR.unpack(_recv_exact(s, _HDR.size))
    return _recv_exact(s, n)


class Rendezvous:
    """Collectives over TCP for `world` ranks; every rank must make the same
    sequence of calls.  world == 1 needs no socket."""

    def __init__(self, rank: int, world: int, addr: str | None = None, port: int | None = None,
                 timeout: float = 300.0):
        self.rank, self.world = int(rank), int(world)
        self._peers: list[socket.socket] = []  # rank 0: sockets of ranks 1..world-1
        self._srv = None
        self._up = None
        if self.world == 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(port or os.environ["MASTER_PORT"])
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            self._srv = socket.socket()
            self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            self._srv.bind((addr, port))
            self._srv.listen(self.world)
            self._srv.settimeout(timeout)
            peers = {}
            while len(peers) < self.world - 1:
                c, _ = self._srv.accept()
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                (r,) = _HDR.unpack(_recv_exact(c, _HDR.size))
                peers[int(r)] = c
            self._peers = [peers[r] for r in range(1, self.world)]
        else:
            while True:
                try:
                    self._up = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            self._up.settimeout(timeout)
            self._up.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._up.sendall(_HDR.pack(self.rank))

    @classmethod
    def from_env(cls, timeout: float = 300.0) -> "Rendezvous":
        world, rank, _ = world_from_env()
        return cls(rank, world, timeout=timeout)

    def _exchange(self, payload: bytes, combine) -> bytes:
        """Rank 0 gathers every rank's payload (rank order), combines them,
        and sends the result back to all."""
        if self.world == 1:
            return combine([payload])
        if self.rank == 0:
            parts = [payload] + [_recv(p) for p in self._peers]
            out = combine(parts)
            for p in self._peers:
                _send(p, out)
            return out
        _send(self._up, payload)
        return _recv(self._up)

    def allreduce(self, values, op: str = "sum") -> np.ndarray:
        v = np.ascontiguousarray(np.atleast_1d(np.asarray(values, np.float64)))
        f = {"sum": np.sum, "max": np.max, "min": np.min}[op]

        def combine(parts):
            arr = np.stack([np.frombuffer(p, np.float64) for p in parts])
            return np.ascontiguousarray(f(arr, axis=0)).tobytes()

        return np.frombuffer(self._exchange(v.tobytes(), combine), np.float64).copy()

    def barrier(self) -> None:
        self.allreduce([0.0])

    def broadcast(self, data: bytes | None) -> bytes:
        """Rank 0's bytes on every rank."""
        return self._exchange(data if self.rank == 0 else b"", lambda parts: parts[0])

    def close(self) -> None:
        for s in self._peers + [self._up, self._srv]:
            if s is not None:
                try:
                    s.close()
                except OSError:
                    pass
        self._peers, self._up, self._srv = [], None, None
