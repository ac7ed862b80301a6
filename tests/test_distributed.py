"""World-size-2 gloo tests of the multi-GPU path's host logic (CPU).

The sharded ICP (realsensetracker_amd/shard.py) splits the
source into contiguous shards, all-reduces the 16 fp64 P2POINT_REF partial
sums once per iteration and solves the same pose on every rank.  Here the
per-shard partial sums come from the oracle (orc_p2point_partials, the same
quantities the GPU kernels reduce) and the exchange is a gloo all-reduce:
the decomposition must reproduce the unsharded fp64-sum loop and every rank
must end on the bitwise-identical pose.  The RCCL unique-id exchange that
sets up the GPU communicator runs for real (ncclGetUniqueId needs no GPU).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden
from oracle import oracle as O
from posemetric import pose_err
from realsensetracker_amd.shard import exchange_unique_id, shard_bounds


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def sharded_icp(src, dst, tree, max_iter, lo, hi, allreduce):
    """P2POINT_REF over shard [lo, hi) with a sum all-reduce of the partials
    (the structure of icp.hip's comm branch)."""
    n = len(src)
    c = np.array([src[lo:hi].astype(np.float64).sum(0).tolist() + [hi - lo]], np.float64)[0]
    c = allreduce(c)
    smean = (c[:3] / c[3]).astype(np.float32)
    T = np.eye(4, dtype=np.float32)
    mu = np.float32(1.0)
    for it in range(max_iter):
        if it > 0 and it % 8 == 0:
            mu = np.float32(mu / np.float32(1.4))
        part = O.p2point_partials(src[lo:hi], tree, T, smean, mu) if hi > lo else np.zeros(16)
        tot = allreduce(part)
        dmean = (tot[12:15] / n).astype(np.float32)
        cov = tot[:9].reshape(3, 3) - dmean.astype(np.float64)[:, None] * tot[9:12][None, :]
        T = O.kabsch_pose(cov, smean, dmean)
    return T


def seq_sum_f32(x):
    """The reference's sequential float32 sum over axis 0 (ascending index)."""
    return np.add.accumulate(np.asarray(x, np.float32), axis=0, dtype=np.float32)[-1]


def sharded_icp_ref(src, dst, tree, max_iter, lo, hi, allgather, allreduce):
    """RST_SUM_REF over shard [lo, hi) (the structure of icp.hip's sharded
    refsum branch): the shards' source and, per iteration, their
    correspondences (q, d2) are all-gathered into the whole source's order,
    every rank takes the reference's sequential fp32 sums over them
    (centroid :85-86, dst_mean :113,122, the same bits on every rank), and
    the covariance of the reference's float products (:125-136) is a
    sharded fp64 sum, all-reduced."""
    n = len(src)
    smean = seq_sum_f32(allgather(src[lo:hi])) * np.float32(1.0 / n)
    T = np.eye(4, dtype=np.float32)
    mu = np.float32(1.0)
    b = (src[lo:hi] - smean).astype(np.float32)
    for it in range(max_iter):
        if it > 0 and it % 8 == 0:
            mu = np.float32(mu / np.float32(1.4))
        if hi > lo:
            idx, d2 = tree.query(O.transform_points(T, src[lo:hi]))
            corr = np.concatenate([dst[idx], d2[:, None]], 1).astype(np.float32)
        else:
            corr = np.zeros((0, 4), np.float32)
        allc = allgather(corr)
        dmean = (seq_sum_f32(allc[:, :3]) / np.float32(n)).astype(np.float32)
        l = (mu / (corr[:, 3] + mu)).astype(np.float32)
        w = (l * l).astype(np.float32)
        a = (w[:, None] * (corr[:, :3] - dmean)).astype(np.float32)
        part = (a[:, :, None] * b[:, None, :]).astype(np.float64).sum(0).ravel()
        cov = allreduce(part).reshape(3, 3)
        T = O.kabsch_pose(cov, smean, dmean)
    return T


def sharded_p2plane(src, tree, normals, max_iter, lo, hi, allreduce, eps=1e-6):
    """The north_star's sharded loop in the point-to-plane mode (the
    structure of icp.hip's comm branch with P2PlaneAcc): each rank's shard
    [lo, hi) gives its 6x6 / 6x1 normal equations (+ count, sum d2), ONE
    all-reduce of those 29 doubles a step, and every rank runs the same
    Cholesky solve and pose update (orc_p2plane_update) -- no broadcast."""
    Rd, td = np.eye(3), np.zeros(3)
    it = 0
    for it in range(1, max_iter + 1):
        part = (O.p2plane_partials(src[lo:hi], tree, normals, Rd, td) if hi > lo else np.zeros(29))
        ok, Rd, td, xn, _ = O.p2plane_update(allreduce(part), Rd, td)
        assert ok
        if xn < eps:
            break
    T = np.eye(4, dtype=np.float32)
    T[:3, :3], T[:3, 3] = Rd.astype(np.float32), td.astype(np.float32)
    return T, it


def _worker(rank, world, port, out, mode="fp64"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        uid = exchange_unique_id()
        ids = [None] * world
        dist.all_gather_object(ids, uid)

        g = load_golden("pair_80x60_s0")
        src, dst = g["src"], g["dst"]
        tree = O.KDTree(dst)
        lo, hi = shard_bounds(len(src), world, rank)

        def allreduce(x):
            t = torch.from_numpy(np.ascontiguousarray(x, np.float64).copy())
            dist.all_reduce(t)
            return t.numpy()

        def allgather(x):  # shards of different lengths, concatenated in rank order
            parts = [None] * world
            dist.all_gather_object(parts, np.ascontiguousarray(x))
            return np.concatenate(parts, 0)

        if mode == "ref":
            T = sharded_icp_ref(src, dst, tree, 32, lo, hi, allgather, allreduce)
        elif mode == "p2plane":
            T, _ = sharded_p2plane(src, tree, O.compute_normals(dst, 16, tree=tree), 30, lo, hi,
                                   allreduce)
        else:
            T = sharded_icp(src, dst, tree, 32, lo, hi, allreduce)
        poses = [None] * world
        dist.all_gather_object(poses, T)
        if rank == 0:
            out.put({"ids": ids, "poses": poses})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_decomposition_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, q), nprocs=world, start_method="spawn",
                       join=True)
    r = q.get()
    assert all(i == r["ids"][0] for i in r["ids"]) and len(r["ids"][0]) == 128
    # every rank solved the bitwise-same pose
    assert all(np.array_equal(p, r["poses"][0]) for p in r["poses"])
    # ... which is the unsharded fp64-sum loop's
    g = load_golden("pair_80x60_s0")
    tree = O.KDTree(g["dst"])
    T1 = sharded_icp(g["src"], g["dst"], tree, 32, 0, len(g["src"]), lambda x: x)
    assert max(pose_err(r["poses"][0], T1)) <= 1e-6
    _, To, _, _ = O.align_icp(g["src"], g["dst"], 32, sum_mode=1)
    assert max(pose_err(T1, To)) <= 2e-5


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_ref_decomposition_gloo(world):
    """The sharded reference-rounding mode: all-gathered correspondences,
    redundant sequential fp32 sums, all-reduced covariance.  Every rank ends
    on the bitwise-same pose, that of the unsharded restatement, within 1e-6
    of the reference-arithmetic oracle (the covariance's fp64 sum order)."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, q, "ref"), nprocs=world, start_method="spawn",
                       join=True)
    r = q.get()
    assert all(np.array_equal(p, r["poses"][0]) for p in r["poses"])
    g = load_golden("pair_80x60_s0")
    tree = O.KDTree(g["dst"])
    T1 = sharded_icp_ref(g["src"], g["dst"], tree, 32, 0, len(g["src"]), lambda x: x, lambda x: x)
    assert max(pose_err(r["poses"][0], T1)) <= 1e-6
    _, To, _, _ = O.align_icp(g["src"], g["dst"], 32, sum_mode=0)
    e = pose_err(T1, To)
    assert max(e) <= 1e-6, e


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_p2plane_decomposition_gloo(world):
    """Point-to-plane sharded as the north_star asks: per iteration one
    all-reduce of the 6x6 / 6x1 normal equations (29 doubles here; 30 on the
    device) over gloo.  Every rank ends on the bitwise-same pose, within 1e-6
    of the unsharded oracle loop (orc_align_p2plane: the same sums in another
    association)."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, q, "p2plane"), nprocs=world,
                       start_method="spawn", join=True)
    r = q.get()
    assert all(np.array_equal(p, r["poses"][0]) for p in r["poses"])
    g = load_golden("pair_80x60_s0")
    tree = O.KDTree(g["dst"])
    nrm = O.compute_normals(g["dst"], 16, tree=tree)
    T1, it1 = sharded_p2plane(g["src"], tree, nrm, 30, 0, len(g["src"]), lambda x: x)
    ito, To, _ = O.align_p2plane(g["src"], g["dst"], nrm, 30, tree=tree)
    assert ito == it1 and ito > 1
    assert np.array_equal(T1, To)  # one shard: orc_align_p2plane's own sums, bit for bit
    e = pose_err(r["poses"][0], To)
    assert max(e) <= 1e-6, e


def test_shard_bounds_tile():
    for n in (0, 1, 5, 7, 307200, 1000001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            sizes = [h - l for l, h in b]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


# ---- RST_SUM_REF sharded by relay ----------------------------------
def _relay_worker(rank, world, port, out, x):
    """Rank r holds the contiguous stretch [lo, hi) of the correspondence
    stream.  One all-gather of the ranks' fp64 totals gives the fp64 prefix
    before the stretch (its guesses' offset); the chain's value at the
    stretch start comes from rank r - 1, the stretch is mapped and walked
    locally (the kernels' arithmetic: tests/cpp/seqsum_emu.cpp), its end goes
    to rank r + 1, and the last rank broadcasts the sums."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path
        sys.path.insert(0, str(Path(__file__).resolve().parent))
        from seqsum_emu import emulate
        lo, hi = shard_bounds(len(x), world, rank)
        mine = x[lo:hi]
        tot = torch.tensor(np.where(np.isfinite(mine), mine, 0).astype(np.float64).sum(0))
        tots = [torch.zeros(4, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(tots, tot)
        p0 = sum((t.numpy() for t in tots[:rank]), np.zeros(4))
        s_in = torch.zeros(4, dtype=torch.float32)
        if rank > 0:
            dist.recv(s_in, src=rank - 1)
        bits, st = emulate(mine, p0=p0, s0=s_in.numpy())
        s_out = torch.from_numpy(bits.view(np.float32).copy())
        if rank + 1 < world:
            dist.send(s_out, dst=rank + 1)
        dist.broadcast(s_out, src=world - 1)
        got = [None] * world
        dist.all_gather_object(got, (s_out.numpy().view(np.uint32).tolist(), st[:, :2].tolist()))
        if rank == 0:
            out.put(got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_ref_sums_relay_gloo(world):
    """The sharded loop's sequential sums without moving correspondences:
    every rank gets the unsharded chain's bits (numpy's sequential float32
    accumulate), and the stretches' superblock maps hit with only the fp64
    prefix as the guesses' offset.  xGMI bytes per iteration: R x 32 B of
    totals, 16 B per relay hop, 16 B broadcast."""
    rng = np.random.default_rng(world)
    n = 120000
    u = np.tile(np.arange(400), n // 400 + 1)[:n]
    x = np.stack([(u - 200) / 385.0 * 2.0, np.full(n, 1.0) + rng.normal(size=n) * 0.1,
                  2.0 + rng.normal(size=n) * 0.01, rng.random(n)], 1).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    mp.start_processes(_relay_worker, args=(world, port, q, x), nprocs=world, start_method="spawn",
                       join=True)
    got = q.get()
    want = np.add.accumulate(np.concatenate([np.zeros((1, 4), np.float32), x]), axis=0,
                             dtype=np.float32)[-1].view(np.uint32).tolist()
    assert all(g[0] == want for g in got), (got, want)
    # (every rank's superblock jumps: most hit with the fp64-prefix guesses.
    # A stretch's first superblock starts from the raw fp64 prefix -- no
    # previous iteration's drift in this one-shot chain -- so each (rank,
    # chain) may miss its first one: at 8 ranks of 15k elements those are a
    # quarter of the tries, 99 / 128 hits measured.  The other superblocks
    # must hit >= 80 %.)
    hits = sum(sum(h for _, h in g[1]) for g in got)
    tries = sum(sum(t for t, _ in g[1]) for g in got)
    first = sum(sum(1 for t, _ in g[1] if t > 0) for g in got)  # one first superblock per walked chain
    assert hits >= 0.8 * (tries - first), (hits, tries, first)
