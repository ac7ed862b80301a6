"""Multi-GPU ICP: the source cloud sharded across ranks (one process per GPU).

The reference has no distribution; this is the build's
scaling of AlignIcp3d (align_icp.cpp:92-153) to one node:

* the target index is replicated (every rank builds it from the same frame);
* the source splits into contiguous shards, ``shard_bounds``;
* RST_SUM_FP64 / RST_P2PLANE: per iteration every rank reduces its 16 / 30
  fp64 partial sums (P2PLANE: the 6x6 / 6x1 normal equations) to one row
  and ONE RCCL all-reduce over xGMI makes them global; every rank then
  solves the same pose (no broadcast);
* the reference-rounding mode (RST_SUM_REF, the library default): the shards
  are contiguous stretches of the source order, and a sequential fp32 sum is
  one chain through them in rank order, so the chains' *values* travel
  instead of the correspondences (comm.hip comm_relay_seqsum): an all-gather
  of each rank's fp64 chain totals (32 B) seeds every rank's maps of its own
  stretch, rank r - 1 sends rank r the exact chain values at its stretch
  start (16 B), rank r walks its stretch and sends the end on, the last rank
  broadcasts the sums (16 B) -- the same bit-exact dst_mean and cost on
  every rank -- and the 9 covariance sums are all-reduced.

Host logic only: the RCCL communicator is created from a unique id that
rank 0 draws and broadcasts -- through ``rendezvous.Rendezvous`` (TCP; what
``bench.py`` uses, no second HIP runtime in the process) or through a
``torch.distributed`` group (the gloo CPU tests).  The per-iteration
exchange is inside librst_align.so (``rst_icp_align_sharded_device``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of n source points for `rank`; shard sizes differ
    by at most one and the shards tile [0, n) in rank order."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError("bad shard spec")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _draw_unique_id() -> bytes:
    raw = C.create_string_buffer(L.COMM_ID_BYTES)
    L.check(L.lib().rst_comm_get_unique_id(raw), "rst_comm_get_unique_id")
    return raw.raw


def exchange_unique_id(group=None, rendezvous=None) -> bytes:
    """Rank 0 draws the RCCL unique id; every rank returns the same bytes
    (over a Rendezvous when given, else a torch.distributed group)."""
    if rendezvous is not None:
        uid = rendezvous.broadcast(_draw_unique_id() if rendezvous.rank == 0 else None)
        assert len(uid) == L.COMM_ID_BYTES
        return uid
    import torch.distributed as dist
    buf = [None]
    if dist.get_rank(group) == 0:
        raw = C.create_string_buffer(L.COMM_ID_BYTES)
        L.check(L.lib().rst_comm_get_unique_id(raw), "rst_comm_get_unique_id")
        buf[0] = raw.raw
    dist.broadcast_object_list(buf, src=0, group=group)
    assert isinstance(buf[0], bytes) and len(buf[0]) == L.COMM_ID_BYTES
    return buf[0]


class ShardedAligner:
    """One rank's side of the sharded ICP.  Every rank calls ``align`` with
    its own shard (device pointer, see ``shard_bounds``) and the replicated
    target; all ranks return the same pose."""

    def __init__(self, ctx, group=None, world: int | None = None, rank: int | None = None,
                 uid: bytes | None = None, rendezvous=None):
        """Ranks from a ``rendezvous.Rendezvous``, from ``torch.distributed``
        (the default), or given explicitly with the RCCL unique id (e.g.
        world 1 without a process group: the id is drawn locally)."""
        self.ctx = ctx
        if rendezvous is not None:
            self.rank, self.world = rendezvous.rank, rendezvous.world
            uid = exchange_unique_id(rendezvous=rendezvous)
        elif world is None:
            import torch.distributed as dist
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
            uid = exchange_unique_id(group)
        else:
            self.world, self.rank = int(world), int(rank or 0)
            if uid is None:
                if self.world != 1:
                    raise ValueError("world > 1 needs the shared unique id")
                raw = C.create_string_buffer(L.COMM_ID_BYTES)
                L.check(L.lib().rst_comm_get_unique_id(raw), "rst_comm_get_unique_id")
                uid = raw.raw
        self._comm = C.c_void_p()
        L.check(L.lib().rst_comm_create(ctx.handle, uid, self.world, self.rank,
                                        C.byref(self._comm)), "rst_comm_create")

    def align(self, d_src_shard: int, n_shard: int, target, opts=None, pose=None,
              n_total: int | None = None):
        """n_total (the points of all shards, when the caller knows it; by
        default opts.n_total): after the communicator's first align, no count
        exchange and no host round trip before the loop.  The library checks
        it against the exchanged shard sizes."""
        pose = np.eye(4, dtype=np.float32) if pose is None else np.asarray(pose, np.float32)
        buf = L.pose_to_cm(pose)
        mc = C.c_float(0)
        o = self._opts(opts, n_total)
        st = L.check(L.lib().rst_icp_align_sharded_device(
            self.ctx.handle, self._comm, C.c_void_p(d_src_shard), int(n_shard), target.handle,
            C.byref(o), L.fptr(buf), C.byref(mc)), "rst_icp_align_sharded_device")
        return st == L.RST_OK, L.cm_to_pose(buf), float(mc.value)

    def align_prepared(self, src_shard, target, opts=None, pose=None, n_total: int | None = None):
        """The same with a prepared source shard (a Target): no per-call
        Morton sort of the shard."""
        pose = np.eye(4, dtype=np.float32) if pose is None else np.asarray(pose, np.float32)
        buf = L.pose_to_cm(pose)
        mc = C.c_float(0)
        o = self._opts(opts, n_total)
        st = L.check(L.lib().rst_icp_align_sharded_prepared(
            self.ctx.handle, self._comm, src_shard.handle, target.handle, C.byref(o),
            L.fptr(buf), C.byref(mc)), "rst_icp_align_sharded_prepared")
        return st == L.RST_OK, L.cm_to_pose(buf), float(mc.value)

    @staticmethod
    def _opts(opts, n_total):
        """A copy of opts (the library defaults when None); n_total only
        overrides opts.n_total when given."""
        o = L.IcpOpts()
        C.memmove(C.byref(o), C.byref(opts if opts is not None else L.default_opts()), C.sizeof(o))
        if n_total is not None:
            o.n_total = int(n_total)
        return o

    def close(self):
        if self._comm:
            L.lib().rst_comm_destroy(self._comm)
            self._comm = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
