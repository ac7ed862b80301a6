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
