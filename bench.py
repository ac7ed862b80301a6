"""Benchmark: ICP iterations/s + frames/s on a 640x480 synthetic RGB-D stream
(BASELINE.json metric, configs[1]).

One step = one batch of --batch (16) incoming frames of the stream, fully on
the GPU, per frame:
    u16 depth (already in HBM) -> unprojection -> Morton sort + BVH build
    (the frame's index, reused as the next pair's target)
    -> AlignIcp3d(curr, prev) with the reference's P2POINT_REF loop,
       128 fixed iterations (rs_replay_app.cpp:246-251),
the batch's 16 frame pairs aligned in lockstep by one
rst_icp_align_batch_async (--batch 0: a step is one frame pair, one align).
value = ICP iterations/s over all ranks (pairs * 128 / time).  Frame
preparation runs on --prep-threads contexts of its own, and --inflight
batches (default 4; 24 HIP hardware queues: --hw-queues) are aligned
concurrently, each on its own context/stream: one batch's iteration chain
is latency-bound, so independent batches overlap on the GPU.  A second timed loop runs the build's point-to-plane mode on the same
frames (reported as extra fields).

The value line runs the drop-in default, RST_SUM_REF: the reference's
sequential fp32 sums exactly as align_icp.cpp rounds them, the mode within
the north_star's 1e-4 gate (24 pairs in flight); the throughput mode
RST_SUM_FP64 (fp64 partial sums, outside that gate) is timed on the same
stream as the extra field "fp64_sums" (--sum-mode fp64 swaps them).

roofline: the dominant kernel k_icp_nn (transform + exact NN + weighted
partial sums of one ICP iteration), algorithmic bytes per launch
12 n + 12 m + S_idx, over its average duration from HIP
events on the aligning stream (every 8th iteration), vs 8 TB/s.  traffic =
HBM bytes per launch from the committed PMC pass (profiles/pmc_*.json:
FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE).  Multi-GPU: one process
per GPU -- `--gpus N` without a launcher spawns the N ranks itself
(realsensetracker_amd/rendezvous.py), or run under torch.distributed.run --
each rank tracks its own stream (frame pairs are independent; no data-path
collective) -> weak scaling; barrier + max-over-ranks timing over a TCP
rendezvous (no torch in the process: the library is its only HIP runtime).

Other BASELINE configs (extra bench lines, same JSON contract):
    --width 1280 --height 720     configs[2]: the stream at 720p
    --mode p2plane                the value leg in the build's point-to-plane mode
                                  to convergence (configs[1-2] name point-to-plane;
                                  the reference's own loop is P2POINT_REF, the default)
    --workload pyramid            configs[4]: 3-level coarse-to-fine ICP on a
                                  1280x720 stream, pose chained on the device
    --workload sharded            configs[3]: a 1000x1000 (~1M-point) pair, the
                                  source sharded over the ranks, one RCCL
                                  all-reduce per iteration (strong scaling)

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import platform
import sys
import time
from collections import deque
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from realsensetracker_amd import _lib as L  # noqa: E402
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402
from realsensetracker_amd import rendezvous as RV  # noqa: E402

METRIC = "ICP iterations/sec + frames/sec, 640×480 RGB-D, 1/2/4/8 MI355X"
# workload -> default frame size (BASELINE.json configs[1] / [4] / [3])
WORKLOADS = {"stream": (640, 480), "pyramid": (1280, 720), "sharded": (1000, 1000)}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def render_frames(seed: int, n: int, K, stride: int):
    """n consecutive frames of the seeded trajectory (the renderer is C++
    behind ctypes, which drops the GIL: a thread pool renders in parallel)."""
    from concurrent.futures import ThreadPoolExecutor
    sc = driver.SyntheticScene(seed)
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        return list(ex.map(lambda i: sc.render(sc.trajectory(i * stride), K,
                                               noise_seed=1000 * seed + i), range(n)))


def pingpong(k: int, n: int) -> int:
    """Frame index k of a stream that runs 0..n-1 and back, so every pair
    is two consecutive trajectory frames (no artificial wrap-around jump)."""
    if n < 2:
        return 0
    p = k % (2 * n - 2)
    return p if p < n else 2 * n - 2 - p


def cpu_baseline(width: int, height: int, iters: int, levels: list | None = None):
    """The oracle's AlignIcp3d restatement (reference arithmetic, own
    nanoflann-style kd-tree) on one frame pair: 1 core (the reference is
    single-threaded), then all cores (OpenMP over the per-point NN loop, the
    sums sequential: same result) as a secondary field.  Sample: the first
    `iters` of the 128 iterations; with `levels` (the pyramid), the same
    coarse-to-fine chain as the GPU on the strided levels, `levels[l]`
    iterations each, counted in level-0 equivalents.  Tree builds are timed
    separately."""
    from oracle import oracle as O
    K = driver.intrinsics(width, height)
    sc = driver.SyntheticScene(0)
    da = sc.render(sc.trajectory(0), K, noise_seed=1)
    db = sc.render(sc.trajectory(1), K, noise_seed=2)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    nlev = len(levels) if levels else 1
    pa = [O.unproject(da, K4, stride=1 << lv) for lv in range(nlev)]
    pb = [O.unproject(db, K4, stride=1 << lv) for lv in range(nlev)]
    t0 = time.perf_counter()
    trees = [O.KDTree(x, 16) for x in pa]
    t1 = time.perf_counter()
    its = levels if levels else [iters]
    eq = sum(its[lv] * len(pb[lv]) / len(pb[0]) for lv in range(nlev))  # level-0 equivalents

    def one():
        T = np.eye(4, dtype=np.float32)
        ts = time.perf_counter()
        for lv in reversed(range(nlev)):
            _, T, _, _ = O.align_icp(pb[lv], pa[lv], its[lv], T=T, tree=trees[lv])
        return time.perf_counter() - ts

    dt1 = one()
    cores = max(1, min(16, os.cpu_count() or 1))
    O.set_threads(cores)
    try:
        dtn = one()
    finally:
        O.set_threads(1)
    what = (f"{nlev}-level pyramid {width}x{height}, iterations {its} (finest first), "
            f"{eq:.1f} level-0-equivalent iterations" if levels else
            f"all {iters} P2POINT_REF iterations" if iters >= 128 else
            f"first {iters} of 128 P2POINT_REF iterations (the early iterations are the "
            f"costliest for a kd-tree: biased low)")
    return {"value": eq / dt1, "unit": "ICP iterations/s", "cores": 1, "kind": "port",
            "sample": f"1 frame pair {width}x{height} (n={len(pb[0])}, m={len(pa[0])}), {what}, "
                      f"oracle/rst_oracle.c -O3, kd-tree leaf 16 prebuilt ({t1 - t0:.3f} s)",
            "seconds": dt1, "cpu": cpu_model(),
            "all_cores": {"value": eq / dtn, "cores": cores, "seconds": dtn,
                          "note": "OpenMP over the per-point NN loop; sums sequential (identical "
                                  "result); secondary baseline, for context"}}


def callers_cpu_baseline(raw, iters: int):
    """The reference callers' sequence (rs_replay_app.cpp:229,246-251) on the
    oracle, 1 core: RemoveNans, DownsampleVoxel 0.05 of both clouds (the
    reference's unordered_map order), AlignIcp3d(curr_down, prev_down, iters)
    with its kd-tree built per call (the 4-argument overload,
    align_icp.cpp:163-167) -- the same frames as the GPU leg, pairs 2-3."""
    from oracle import oracle as O
    O.set_threads(1)
    ts, npts = [], []
    for k in (2, 3):
        t0 = time.perf_counter()
        cur = O.downsample_voxel(O.remove_nans(raw[k]), 0.05)
        prv = O.downsample_voxel(O.remove_nans(raw[k - 1]), 0.05)
        O.align_icp(cur, prv, iters, tree=O.KDTree(prv, 16))
        ts.append(time.perf_counter() - t0)
        npts.append(len(cur))
    ms = 1000.0 * float(np.mean(ts))
    return {"ms_per_pair": ms, "iterations_per_s": iters / (ms * 1e-3), "cores": 1, "kind": "port",
            "points_per_cloud": int(np.mean(npts)), "cpu": cpu_model(),
            "sample": f"2 frame pairs of the callers' workload, {iters} P2POINT_REF iterations each, "
                      "oracle/rst_oracle.c -O3 (reference arithmetic, nanoflann-style kd-tree "
                      "leaf 16 built per call), preprocessing included"}


DEFAULT_CONFIG = "stream_640x480_p2point_ref"


def load_traffic(config: str = DEFAULT_CONFIG):
    """HBM bytes per pair iteration of the NN pass (k_icp_nn + k_icp_fb, or
    a batched launch's share per pair) from a
    committed PMC summary (profiles/pmc_*.json, scripts/pmc_traffic.py) of
    this workload (`config`: workload_WxH_mode; summaries without one are of
    the default) -- only one stamped with this library's source hash
    (lib/BUILD_INFO.json): a pass of other code is not reported.  Returns
    (bytes | None, origin)."""
    try:
        cur = json.loads((ROOT / "realsensetracker_amd" / "lib" / "BUILD_INFO.json").read_text())
        cur = cur.get("source_hash")
    except (OSError, ValueError):
        cur = None
    for f in sorted(ROOT.glob("profiles/pmc_*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        if (cur and d.get("source_hash") == cur and "nn_pass_bytes_per_pair_iteration" in d and
                d.get("config", DEFAULT_CONFIG) == config):
            return d["nn_pass_bytes_per_pair_iteration"], f.name
    return None, f"no PMC pass of this build (source hash {cur}) of {config} under profiles/"


def p2point_alg_bytes(n: float, m: float) -> float:
    """SURVEY.md §8d fused P2POINT iteration: 12 n + 12 m + S_idx, S_idx =
    leaf boxes (64 B) + leaf ranges (4 B) of the power-of-two leaf count."""
    nleaves = 1
    while nleaves * 16 < m:
        nleaves *= 2
    return 12 * n + 12 * m + 64 * nleaves + 4 * (nleaves + 1)


def pyramid_level_roofline(a, d_depth, K, nfr, c, pctx, opts, normals_k, pyr_iters):
    """configs[4]'s roofline per level: each level's NN pass (k_icp_nn +
    k_icp_fb) -- its algorithmic bytes (SURVEY.md §8d with that level's n, m)
    over its own average kernel time (HIP events around every iteration) --
    over --roof-steps frame pairs, the levels aligned coarsest first with the
    pose chained, as rst_icp_align_pyramid_async runs them."""
    out = [{"level": lv, "iters": pyr_iters[lv], "n": 0, "m": 0, "nn_us": 0.0, "launches": 0}
           for lv in range(a.levels)]
    c.enable_kernel_timing(1)
    try:
        for k in range(1, a.roof_steps + 1):
            cur = A.Target.pyramid_from_depth_device(d_depth[pingpong(k, nfr)].value, K, a.levels,
                                                     normals_k, pctx)
            prv = A.Target.pyramid_from_depth_device(d_depth[pingpong(k - 1, nfr)].value, K,
                                                     a.levels, normals_k, pctx)
            pctx.synchronize()
            pose = np.eye(4, dtype=np.float32)
            for lv in reversed(range(a.levels)):
                o = L.default_opts(max_iter=pyr_iters[lv], sum_mode=opts.sum_mode, mode=opts.mode)
                r = A.align_prepared_async(cur[lv], prv[lv], c, pose, o).wait()
                it3, nl = c.last_iteration_times()
                x = out[lv]
                x["n"] += len(cur[lv])
                x["m"] += len(prv[lv])
                x["nn_us"] += 1000.0 * (it3[0] + it3[1]) * nl
                x["launches"] += nl
                if r.ok:
                    pose = r.pose
            for t in cur + prv:
                t.free()
    finally:
        c.enable_kernel_timing(0)
    for x in out:
        f = max(1, a.roof_steps)
        x["n"] /= f
        x["m"] /= f
        x["nn_us"] /= max(1, x["launches"])
        x["alg_bytes"] = p2point_alg_bytes(x["n"], x["m"])
        x["achieved_GBps"] = x["alg_bytes"] / (x["nn_us"] * 1e-6) / 1e9 if x["nn_us"] > 0 else 0.0
        x["frac"] = x["achieved_GBps"] / HBM_PEAK_GBS
    return out


SHARDED_MODES = {  # --workload sharded --mode / --sum-mode -> the align's options
    "ref": ("RST_SUM_REF: the reference's sequential fp32 sums, bit-exact (within the 1e-4 gate)",
            "per iteration the sequential fp32 sums relayed rank to rank (an all-gather of 32 B "
            "fp64 totals per rank, 16 B chain values sent on, a 16 B broadcast; each rank maps "
            "and walks its own stretch), one all-reduce of 9 fp64"),
    "fp64": ("RST_SUM_FP64: fp64 partial sums (outside the 1e-4 gate of the reference's fp32 "
             "sums: tests/golden/fp64_gate.json)", "one RCCL all-reduce of 16 fp64 per iteration"),
    "p2plane": ("fp64 6x6 / 6x1 point-to-plane normal equations (absent in the reference, "
                "SURVEY.md §8 a11), image-grid normals",
                "one RCCL all-reduce of the 30-double normal equations per iteration (the "
                "north_star's split), every rank the same Cholesky solve"),
}


def sharded_leg(kind: str, width: int, height: int, iters: int, steps: int, warmup: int,
                frames_dev, local: int, rank: int, world: int, rdv, barrier, max_over_ranks,
                hip, K=None):
    """configs[3]: one large scan pair (default 1000x1000 depth, ~1M points),
    the source sharded across the ranks (contiguous point ranges of its
    original order, shard_bounds), the target index replicated; per
    iteration the exchange of `kind` (SHARDED_MODES) over RCCL / xGMI
    (rst_icp_align_sharded_device).  A step = one AlignIcp3d of the pair
    (`iters` iterations; point-to-plane to convergence, <= 30); total work is
    fixed as N grows (strong scaling).  frames_dev: the two depth frames in
    HBM (target, source).  Returns the timing dict (every rank; timing is
    max over ranks)."""
    from realsensetracker_amd.shard import ShardedAligner, shard_bounds
    K = K or driver.intrinsics(width, height)
    ctx = A.Context(local)
    plane = kind == "p2plane"
    tgt = A.Target.from_depth_device(frames_dev[0].value, K, -2 if plane else 0, ctx)
    d_src = C.c_void_p()
    assert hip.hipMalloc(C.byref(d_src), C.c_size_t(12 * width * height)) == 0
    n = C.c_int64(0)
    L.check(L.lib().rst_unproject_device(ctx.handle, frames_dev[1], C.byref(K), 0, d_src,
                                         C.byref(n)), "rst_unproject_device")
    lo, hi = shard_bounds(n.value, world, rank)
    sh = ShardedAligner(ctx, rendezvous=rdv)
    if plane:
        opts = L.default_opts(mode=L.RST_P2PLANE, max_iter=30)
    else:
        opts = L.default_opts(max_iter=iters,
                              sum_mode=L.RST_SUM_REF if kind == "ref" else L.RST_SUM_FP64)
    ptr = d_src.value + 12 * lo
    try:
        def step():  # every rank knows the global count: no host round trip per align
            ok, pose, _ = sh.align(ptr, hi - lo, tgt, opts, n_total=n.value)
            return ok, pose

        for _ in range(warmup):
            step()
        ctx.enable_kernel_timing(8)
        kms, kl, oks, its = 0.0, 0, 0, 0
        barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        pose = np.eye(4, dtype=np.float32)
        for _ in range(steps):
            ok, pose = step()
            oks += int(ok)
            its += ctx.last_iterations()  # (point-to-plane: to convergence; every rank alike)
            ms, nl = ctx.last_kernel_time()
            kms += ms * nl
            kl += nl
        ctx.synchronize()
        barrier()
        dt = max_over_ranks(time.perf_counter() - t0)
        ctx.enable_kernel_timing(0)
        it_pair = its / max(1, steps)
        avg_ms = kms / max(1, kl)
        alg = p2point_alg_bytes(hi - lo, len(tgt)) + (12 * len(tgt) if plane else 0)
        achieved = alg / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        return {"kind": kind, "value": its / dt, "unit": "ICP iterations/s",
                "n_ranks": world, "steps": steps, "warmup": warmup,
                "ms_per_step": 1000.0 * dt / steps, "iters_per_pair": it_pair,
                "points": n.value, "target_points": len(tgt), "shard_points": hi - lo,
                "pairs_ok": oks, "final_pose_t": [float(x) for x in pose[:3, 3]],
                "accumulation": SHARDED_MODES[kind][0], "exchange": SHARDED_MODES[kind][1],
                "nn_avg_us": 1000.0 * avg_ms, "alg_bytes_per_launch": alg,
                "achieved_GBps": achieved}
    finally:
        sh.close()
        tgt.free()
        hip.hipFree(d_src)
        ctx.close()


def run_sharded(a, K, frames, d_depth, hip, world, rank, local, rdv, barrier, max_over_ranks):
    """configs[3] as the bench line (--workload sharded): value = the pair's
    ICP iterations/s with the source sharded over the ranks (sharded_leg)."""
    kind = "p2plane" if a.mode == "p2plane" else a.sum_mode
    r = sharded_leg(kind, a.width, a.height, a.iters, a.steps, a.warmup, d_depth, local, rank,
                    world, rdv, barrier, max_over_ranks, hip, K)
    if rank == 0:
        cpu = None if a.no_cpu or world > 1 else cpu_baseline(a.width, a.height, a.cpu_iters)
        value = r["value"]
        out = {
            "metric": METRIC, "value": value, "unit": "ICP iterations/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": r["ms_per_step"],
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded procedural room, ray-cast u16 depth, 1 mm noise, "
                    "~3% invalid)",
            "config": {"workload": f"{a.width}x{a.height} scan pair ({r['points']} source points), "
                                   + ("point-to-plane to convergence (<= 30 iters)"
                                      if kind == "p2plane" else
                                      f"AlignIcp3d P2POINT_REF {a.iters} iters")
                                   + f", source sharded over {world} rank(s), " + r["exchange"],
                       "width": a.width, "height": a.height, "iters_per_pair": r["iters_per_pair"],
                       "points_per_frame": r["points"], "target_points": r["target_points"],
                       "mode": "P2PLANE" if kind == "p2plane" else "P2POINT_REF",
                       "accumulation": r["accumulation"],
                       "parallelism": f"shard{world}"},
            "frames_per_s": a.steps / (r["ms_per_step"] * a.steps * 1e-3), "pairs_ok": r["pairs_ok"],
            "final_pose_t": r["final_pose_t"],
            "roofline": {"bound": "hbm", "achieved": r["achieved_GBps"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": r["achieved_GBps"] / HBM_PEAK_GBS,
                         "traffic": None, "kernel": "k_icp_nn+k_icp_fb (rank 0's shard)",
                         "avg_us": r["nn_avg_us"],
                         "alg_bytes_per_launch": r["alg_bytes_per_launch"]},
            "cpu_baseline": cpu,
        }
        if cpu is not None:
            out["speedup_vs_cpu_baseline"] = value / cpu["value"]
        print(json.dumps(out))
    rdv.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20,
                    help="timed steps: batches of --batch frame pairs (one frame pair each with "
                         "--batch 0, and for the pyramid / point-to-plane / sharded workloads)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="stream",
                    help="stream: configs[1] (configs[2] with --width 1280 --height 720); "
                         "pyramid: configs[4]; sharded: configs[3]")
    ap.add_argument("--width", type=int, default=0, help="0: the workload's default")
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--levels", type=int, default=3, help="pyramid levels (stride 2^l)")
    ap.add_argument("--pyr-iters", default="32,32,64",
                    help="pyramid: P2POINT_REF iterations per level, finest first")
    ap.add_argument("--frames", type=int, default=0,
                    help="distinct frames per rank (0: one per step, at most 512)")
    ap.add_argument("--stride", type=int, default=1, help="trajectory frames between frames")
    ap.add_argument("--iters", type=int, default=128)
    ap.add_argument("--no-p2plane", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=128,
                    help="CPU baseline sample: the first N of the pair's 128 iterations (all "
                         "128 by default: the early iterations are the costliest for a kd-tree)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-api", action="store_true")
    ap.add_argument("--no-gicp", action="store_true")
    ap.add_argument("--graphs", action="store_true",
                    help="replay each align's iteration loop as a hipGraph (no kernel timing)")
    ap.add_argument("--mode", choices=["p2point_ref", "p2plane"], default="p2point_ref",
                    help="the value leg's ICP: the reference's loop (AlignIcp3d P2POINT_REF, "
                         "--iters fixed iterations) or the build's point-to-plane mode to "
                         "convergence (<= 30 iterations, image-grid normals; BASELINE configs[1-2] "
                         "name point-to-plane)")
    ap.add_argument("--sum-mode", choices=["fp64", "ref"], default="ref",
                    help="the value leg's sums: fp64 = RST_SUM_FP64 (fp64 partial sums), "
                         "ref = RST_SUM_REF (the drop-in default: the reference's sequential "
                         "fp32 sums, bit-exact); the other mode is timed as an extra field")
    ap.add_argument("--inflight", type=int, default=0,
                    help="aligns in flight per GPU, one HIP stream each (a batched align "
                         "carries --batch pairs); 0: 4 batched, else 4 in the fp64 mode and "
                         "--ref-inflight in the ref mode")
    ap.add_argument("--hw-queues", type=int, default=24,
                    help="GPU_MAX_HW_QUEUES for this process (HIP's default, 4, puts the "
                         "frame-preparation stream and 4 pairs' streams on 4 hardware queues; "
                         "r02u/v: 2 pairs 16.2k, 4 pairs 15.8k it/s at 4 queues, 19.4k at 8; "
                         "r02m: one queue per stream of the reference-rounding leg too "
                         "(24 pairs: 7.1k vs 3.0k it/s at 8 queues, main leg unchanged); "
                         "0: leave the environment's value)")
    ap.add_argument("--ref-steps", type=int, default=-1,
                    help="frame pairs timed in the other sum mode (extra field; -1: as many as "
                         "the value leg, 0: skip)")
    ap.add_argument("--ref-inflight", type=int, default=24,
                    help="frame pairs in flight in the reference-rounding leg: its sequential "
                         "sums run one wavefront per component for most of an iteration, so "
                         "more pairs share the GPU")
    ap.add_argument("--batch", type=int, default=-1,
                    help="frame pairs per batched align (rst_icp_align_batch_async: one launch of "
                         "each loop kernel for the whole batch, r06h: 8 x 4 in flight 23.0k it/s "
                         "vs 15.1k for 24 single aligns; r11 shape sweep, 480 pairs: 8 x 4 "
                         "31.95k, 10 x 4 32.5k, 12 x 4 32.6k, 16 x 3 32.4k; r15 build, 480 pairs: "
                         "12 x 4 35.2k, 16 x 4 36.0k, 16 x 3 34.9k, 20 x 3 35.1k, 12 x 5 33.4k; "
                         "720p: 8 8.9k, 12 9.4k, 16 8.1k); 0 = one pair per align; default 16 "
                         "up to 640x480, 12 above")
    ap.add_argument("--prep-threads", type=int, default=3,
                    help="frame-preparation contexts / host threads of the batched legs (each "
                         "frame's unproject + index build is host-synchronous; r10 one context)")
    ap.add_argument("--no-sharded", action="store_true",
                    help="skip the stream line's sharded_1M field (configs[3] over all ranks)")
    ap.add_argument("--sharded-steps", type=int, default=5,
                    help="timed aligns of each sharded_1M mode")
    ap.add_argument("--sharded-timeout", type=float, default=120.0,
                    help="watchdog of the sharded_1M field (s)")
    ap.add_argument("--roof-steps", type=int, default=4,
                    help="frames of the one-pair-in-flight kernel timing pass (roofline; "
                         "batched: the value leg's --steps pairs, one batch in flight)")
    a = ap.parse_args()
    if a.hw_queues > 0:  # read by the HIP runtime at its first call (none yet)
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # no launcher: one rank process per GPU, spawned before any GPU call
        return RV.launch(a.gpus, sys.argv[1:], str(Path(__file__).resolve()))
    dw, dh = WORKLOADS[a.workload]
    a.width, a.height = a.width or dw, a.height or dh
    if a.batch < 0:  # (a batch's points: 16 VGA frames, 12 at 720p -- the sweeps above)
        a.batch = 16 if a.width * a.height <= 640 * 480 else 12
    pyr = a.workload == "pyramid"
    pyr_iters = [int(x) for x in a.pyr_iters.split(",")] if pyr else [a.iters]
    if pyr and len(pyr_iters) != a.levels:
        ap.error("--pyr-iters needs one count per level")

    world, rank, local = RV.world_from_env()
    if world > 1 and a.gpus != world:
        ap.error(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    rdv = RV.Rendezvous(rank, world)  # barrier / timing only, no data path

    def barrier():
        rdv.barrier()

    def max_over_ranks(x: float) -> float:
        return float(rdv.allreduce([x], "max")[0])

    def sum_over_ranks(x: float) -> float:
        return float(rdv.allreduce([x], "sum")[0])

    K = driver.intrinsics(a.width, a.height)
    batched = a.batch > 0 and not pyr and a.workload == "stream"
    pps = a.batch if batched else 1  # frame pairs per step
    npairs = a.steps * pps  # timed pairs
    nfr = max(2, a.frames if a.frames > 0 else min(512, max(npairs, a.warmup * pps) + 1))
    if a.workload == "sharded":
        nfr = 2  # one pair, aligned every step
    frames = render_frames(seed=rank, n=nfr, K=K, stride=a.stride)
    # depth frames resident in HBM before timing (hipMalloc'd via ctypes)
    hip = C.CDLL("libamdhip64.so")
    npx = a.width * a.height
    d_depth = []
    for f in frames:
        p = C.c_void_p()
        assert hip.hipSetDevice(local) == 0
        assert hip.hipMalloc(C.byref(p), C.c_size_t(2 * npx)) == 0
        assert hip.hipMemcpy(p, f.ctypes.data_as(C.c_void_p), C.c_size_t(2 * npx), 1) == 0
        d_depth.append(p)

    if a.workload == "sharded":
        return run_sharded(a, K, frames, d_depth, hip, world, rank, local, rdv, barrier,
                           max_over_ranks)

    opts_fp64 = L.default_opts(max_iter=a.iters, sum_mode=L.RST_SUM_FP64)
    opts_exact = L.default_opts(max_iter=a.iters, sum_mode=L.RST_SUM_REF)
    main_ref = a.sum_mode == "ref"
    opts_main, opts_other = (opts_exact, opts_fp64) if main_ref else (opts_fp64, opts_exact)
    if a.inflight <= 0:
        a.inflight = 4 if batched or not main_ref else a.ref_inflight
    opts_pl = L.default_opts(mode=L.RST_P2PLANE, max_iter=30)
    plane = a.mode == "p2plane"
    nk_main = -2 if plane else 0  # the value leg's normals (image-grid PCA 5x5 for P2PLANE)
    if plane:
        opts_main = opts_pl
        a.ref_steps = 0  # (the sum modes are the point-to-point loop's)
        a.no_p2plane = True  # (the value is that leg)
    # frame preparation on its own context (stream); each frame pair in
    # flight on its own context, so the latency-bound per-iteration chains
    # of independent pairs overlap on the GPU
    pctx = A.Context(local)
    actx = [A.Context(local) for _ in range(max(1, a.inflight))]
    # frame preparation (unproject + index build, host-synchronous per frame)
    # on --prep-threads contexts and host threads, so a batch's frames are
    # prepared in parallel and ahead of the aligns that use them
    import queue
    from concurrent.futures import ThreadPoolExecutor
    prep_ctxs = [pctx] + [A.Context(local) for _ in range(max(0, a.prep_threads - 1))]
    prep_free: "queue.Queue" = queue.Queue()
    for c_ in prep_ctxs:
        prep_free.put(c_)
    prep_pool = ThreadPoolExecutor(max_workers=len(prep_ctxs))

    def run(nsteps: int, opts, normals_k: int, stats: dict | None, ctxs=None):
        ctxs = ctxs or actx
        pending = deque()

        def prep(f):  # frame -> its level targets (one level unless pyramid), on a
            # free preparation context (one host thread each)
            pc = prep_free.get()
            try:
                if pyr:
                    return A.Target.pyramid_from_depth_device(d_depth[f].value, K, a.levels,
                                                              normals_k, pc)
                return [A.Target.from_depth_device(d_depth[f].value, K, normals_k, pc)]
            finally:
                prep_free.put(pc)

        def finish_one():
            pa, c, cur, tgt = pending.popleft()
            r = pa.wait()
            if stats is not None:
                # pyramid P2POINT_REF: every level runs its fixed count; a coarse
                # level's iteration is worth n_l / n_0 of a level-0 one
                coarse = lv_iters[1:] if pyr and opts.mode == L.RST_P2POINT_REF else []
                stats["iters"] += r.iterations + sum(
                    it * len(cur[lv + 1]) / max(1, len(cur[0])) for lv, it in enumerate(coarse))
                stats["iters_all"] += r.iterations + sum(coarse)
                stats["n"] += len(cur[0])
                stats["m"] += len(tgt[0])
                stats["ok"] += int(r.ok)
                ms, nl = c.last_kernel_time()
                stats["kernel_ms"] += ms * nl
                stats["launches"] += nl
                if nl:
                    it3, _ = c.last_iteration_times()
                    for k in range(3):
                        stats["iter_ms"][k] += it3[k] * nl
            for t in tgt:  # frame f: target of pair f, source of pair f-1 (done)
                t.free()

        lv_iters = pyr_iters if opts.mode == L.RST_P2POINT_REF else [opts.max_iter] * a.levels
        prev = prep(0)
        k = 1
        # the frames of the next steps prepared ahead, in parallel
        ahead = deque(prep_pool.submit(prep, pingpong(1 + j, nfr))
                      for j in range(min(len(prep_ctxs), nsteps)))
        for s in range(nsteps):
            cur = ahead.popleft().result()
            if s + len(ahead) + 1 < nsteps:
                ahead.append(prep_pool.submit(prep, pingpong(s + len(ahead) + 2, nfr)))
            if len(pending) == len(ctxs):
                finish_one()
            c = ctxs[s % len(ctxs)]
            # AlignIcp3d(curr, prev, 128, &xfm), xfm = Identity (rs_replay_app.cpp:235,251)
            if pyr:
                pa = A.align_pyramid_async(cur, prev, c, lv_iters, None, opts)
            else:
                pa = A.align_prepared_async(cur[0], prev[0], c, None, opts)
            pending.append((pa, c, cur, prev))
            prev = cur
            k += 1
        while pending:
            finish_one()
        for t in prev:
            t.free()

    def run_batched(nsteps: int, opts, normals_k: int, stats: dict | None, ctxs, B: int):
        # B consecutive frame pairs per align call, in lockstep (one launch of
        # each loop kernel covers the batch); len(ctxs) batches in flight
        pending = deque()

        def prep_job(f):  # on a free preparation context (one thread each)
            pc = prep_free.get()
            try:
                return A.Target.from_depth_device(d_depth[f].value, K, normals_k, pc)
            finally:
                prep_free.put(pc)

        def submit(k0, nb):  # the frames of a batch, prepared in parallel
            return [prep_pool.submit(prep_job, pingpong(k0 + j, nfr)) for j in range(nb)]

        def finish_one():
            pb, c, curs, prevs = pending.popleft()
            rs = pb.wait()
            if stats is not None:
                ms, nl = c.last_kernel_time()
                stats["kernel_ms"] += ms * nl
                stats["launches"] += nl
                if nl:
                    it3, _ = c.last_iteration_times()
                    for k in range(3):
                        stats["iter_ms"][k] += it3[k] * nl
                stats["batches"] += 1
                stats["batch_pairs"] += len(rs)
                for r, cur, tg in zip(rs, curs, prevs):
                    stats["iters"] += r.iterations
                    stats["iters_all"] += r.iterations
                    stats["n"] += len(cur)
                    stats["m"] += len(tg)
                    stats["ok"] += int(r.ok)
            for tg in prevs:  # each a target here and a source of a finished pair
                tg.free()

        prev = prep_job(0)
        k, s, nbatch = 1, 0, 0
        futs = submit(k, min(B, nsteps))
        while s < nsteps:
            nb = min(B, nsteps - s)
            curs, prevs = [], []
            for fu in futs:
                cur = fu.result()
                curs.append(cur)
                prevs.append(prev)
                prev = cur
                k += 1
            # the next batch's frames are prepared (other streams, host threads)
            # while this thread waits for the GPU below
            futs = submit(k, min(B, nsteps - s - nb)) if s + nb < nsteps else []
            if len(pending) == len(ctxs):
                finish_one()
            c = ctxs[nbatch % len(ctxs)]
            # AlignIcp3d(curr, prev, 128, &xfm), xfm = Identity per pair (rs_replay_app.cpp:235,251)
            pending.append((A.align_batch_async(curs, prevs, c, None, opts), c, curs, prevs))
            s += nb
            nbatch += 1
        while pending:
            finish_one()
        prev.free()

    def new_stats():
        return {"iters": 0.0, "iters_all": 0, "n": 0, "m": 0, "ok": 0, "kernel_ms": 0.0,
                "launches": 0, "iter_ms": [0.0, 0.0, 0.0], "batches": 0, "batch_pairs": 0}

    if a.graphs:
        for c in actx:
            c.enable_graphs(True)

    def timing(on, ctxs=None):
        for c in ctxs or actx:  # HIP events in each (every `on`-th) iteration
            c.enable_kernel_timing(0 if a.graphs else int(on))

    def sync_all():
        for c in prep_ctxs + actx:
            c.synchronize()

    # ---- throughput mode (value): no events in the timed region -----------------
    # warm-up: W steps, and at least one per context in flight, so that no
    # context sizes its device workspace inside the timed region
    warm_steps = max(a.warmup, len(actx))
    if batched:
        run_batched(warm_steps * a.batch, opts_main, nk_main, None, actx, a.batch)
    else:
        run(warm_steps, opts_main, nk_main, None)
    st = new_stats()
    barrier()
    sync_all()
    t0 = time.perf_counter()
    if batched:
        run_batched(npairs, opts_main, nk_main, st, actx, a.batch)
    else:
        run(npairs, opts_main, nk_main, st)
    sync_all()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    iters_all = sum_over_ranks(st["iters"])
    iters_raw = sum_over_ranks(st["iters_all"])  # pyramid: every level's iteration counted once
    frames_all = sum_over_ranks(npairs)

    # ---- roofline: one pair in flight, events around every iteration's kernels --
    # (with two pairs in flight an event span also counts the CUs the other
    # pair holds; alone, the spans agree with rocprof's kernel durations)
    # (under --graphs the timing pass runs its one context in stream mode:
    # events cannot sit inside a replayed graph)
    # (batched: one batch in flight, its launches cover the batch's pairs; the
    # value leg's frame pairs -- the same full batches --, whose difficulty
    # varies along the trajectory: r06 first 8 pairs nn+fb 281 us, pairs 25-32
    # 126 us per batched launch)
    sr1 = new_stats()
    actx[0].enable_kernel_timing(1)  # (a timed align runs in stream mode)
    if batched:
        run_batched(npairs, opts_main, nk_main, sr1, actx[:1], a.batch)
    else:
        run(a.roof_steps, opts_main, nk_main, sr1, ctxs=actx[:1])
    actx[0].enable_kernel_timing(0)

    # ---- point-to-plane mode (extra fields) ---------------------------------------
    def p2plane_leg(normals_k: int) -> dict:
        # 4 aligns in flight, batched as the value leg (--batch pairs each) unless
        # --batch 0: a ~7-iteration pair is bound by its frame's preparation,
        # which a deeper queue of aligns only delays
        pctxs = actx[:4]
        B = a.batch if a.batch > 0 else 0
        np_pl = max(a.steps * max(1, B), 8)

        def go(k, stats):
            if B:
                run_batched(k, opts_pl, normals_k, stats, pctxs, B)
            else:
                run(k, opts_pl, normals_k, stats, pctxs)
        go(max(a.warmup, len(pctxs)) * max(1, B), None)
        timing(8, pctxs)
        sp = new_stats()
        barrier()
        sync_all()
        t1 = time.perf_counter()
        go(np_pl, sp)
        sync_all()
        barrier()
        timing(0, pctxs)
        dtp = max_over_ranks(time.perf_counter() - t1)
        return {"iterations_per_s": sum_over_ranks(sp["iters"]) / dtp,
                "pairs_in_flight": len(pctxs) * max(1, B), "pairs_per_batch": max(1, B),
                "pairs": np_pl, "frames_per_s": sum_over_ranks(np_pl) / dtp,
                "mean_iterations_per_pair": sp["iters"] / max(1, np_pl),
                "ms_per_pair": 1000.0 * dtp / np_pl,
                "k_p2plane_avg_us": 1000.0 * sp["kernel_ms"] / max(1, sp["launches"]),
                "normals": ("image-grid PCA, %dx%d window (rst_target_compute_grid_normals)"
                            % (1 - 2 * normals_k, 1 - 2 * normals_k)) if normals_k < 0 else
                           "kNN-%d PCA (ComputeNormals, point_cloud_utils.cpp:176-216)" % normals_k}

    pl = None
    if not a.no_p2plane:
        # perf mode: image-grid normals; the reference's kNN-16 normals beside it
        pl = p2plane_leg(-2)
        pl["knn16_normals"] = p2plane_leg(16)

    # ---- the other sum mode (extra field, not value) -----------------------------
    # fp64 value leg: RST_SUM_REF (the drop-in default) as "ref_sums"; ref value
    # leg: RST_SUM_FP64 as "fp64_sums"
    refs = None
    if a.ref_steps < 0:
        a.ref_steps = npairs
    if a.ref_steps > 0 and not pyr:
        n_other = 4 if main_ref or batched else a.ref_inflight
        rctx = (actx + [A.Context(local) for _ in range(max(0, n_other - len(actx)))])[:n_other]
        if batched:
            run_batched(len(rctx) * a.batch, opts_other, 0, None, rctx, a.batch)
        else:
            run(len(rctx), opts_other, 0, None, rctx)  # every context warmed (as above)
        sr = new_stats()
        barrier()
        sync_all()
        t4 = time.perf_counter()
        if batched:
            run_batched(a.ref_steps, opts_other, 0, sr, rctx, a.batch)
        else:
            run(a.ref_steps, opts_other, 0, sr, rctx)
        sync_all()
        barrier()
        dtr = max_over_ranks(time.perf_counter() - t4)
        refs = {"iterations_per_s": sum_over_ranks(sr["iters"]) / dtr,
                "frames_per_s": sum_over_ranks(a.ref_steps) / dtr,
                "ms_per_pair": 1000.0 * dtr / a.ref_steps, "steps": a.ref_steps,
                "pairs_in_flight": len(rctx) * (a.batch if batched else 1),
                "pairs_per_batch": a.batch if batched else 1,
                "pairs_ok": sr["ok"],
                "note": ("RST_SUM_FP64 (throughput mode, not the drop-in default): fp64 "
                         "partial sums, pose within 2e-5 of the fp64-sum oracle but not "
                         "within the 1e-4 gate of the reference's fp32 sums"
                         if main_ref else
                         "RST_SUM_REF (library default): source centroid, dst_mean and cost "
                         "as sequential fp32 sums in source order, the reference's rounding "
                         "(align_icp.cpp:113,120-122; point_cloud_utils.cpp:92-98)")}

    # ---- the reference-shaped host API (extra fields, not value) ------------------
    # AlignIcp3d(src, dst, 128, &T) on host clouds, one pair at a time: PCIe
    # upload of both clouds + index build + 128 iterations + pose readback
    host = None
    if not a.no_host_api and not pyr:
        clouds = [driver.unproject(frames[pingpong(k, nfr)], K) for k in range(4)]
        T = np.eye(4, dtype=np.float32)
        A.AlignIcp3d(clouds[1], clouds[0], a.iters, T)  # warm the context's pools
        t2 = time.perf_counter()
        for k in range(1, 4):
            T = np.eye(4, dtype=np.float32)
            A.AlignIcp3d(clouds[k], clouds[k - 1], a.iters, T)
        dth = (time.perf_counter() - t2) / 3
        host = {"ms_per_pair": 1000.0 * dth, "pairs_per_s": 1.0 / dth,
                "iterations_per_s": a.iters / dth,
                "sum_mode": "RST_SUM_REF (the drop-in default)",
                "note": "AlignIcp3d(src, dst, 128, T) with host clouds, one pair at a time: "
                        "PCIe-inclusive (upload, index build, ICP, readback)"}

    # ---- the reference callers' own workload (extra fields) ----------------------
    # rs_replay_app.cpp:229,246-251 per frame: RemoveNans(cloud_raw) ->
    # DownsampleVoxel(curr, 0.05) and DownsampleVoxel(prev, 0.05) ->
    # AlignIcp3d(curr_down, prev_down, 128, &xfm) (the 4-argument overload:
    # the target's index built per call), host clouds, one pair at a time
    callers = None
    if not a.no_host_api and not pyr:
        raw = [driver.unproject(frames[pingpong(k, nfr)], K, keep_invalid=True) for k in range(5)]
        callers = {}
        for name, sm in (("ref_sums", L.RST_SUM_REF), ("fp64_sums", L.RST_SUM_FP64)):
            o = L.default_opts(sum_mode=sm)

            ph = [0.0, 0.0]  # prepare (RemoveNans + DownsampleVoxel of both), align

            def pair(k):
                t = time.perf_counter()
                cur = A.DownsampleVoxel(A.RemoveNans(raw[k]), 0.05)
                prv = A.DownsampleVoxel(A.RemoveNans(raw[k - 1]), 0.05)
                t2 = time.perf_counter()
                T = np.eye(4, dtype=np.float32)
                A.AlignIcp3d(cur, prv, a.iters, T, opts=o)
                ph[0] += t2 - t
                ph[1] += time.perf_counter() - t2
                return len(cur)

            pair(1)  # warm the context's pools
            ph[0] = ph[1] = 0.0
            t5 = time.perf_counter()
            npts = [pair(k) for k in range(2, 5)]
            dtc = (time.perf_counter() - t5) / 3
            callers[name] = {"ms_per_pair": 1000.0 * dtc, "pairs_per_s": 1.0 / dtc,
                             "iterations_per_s": a.iters / dtc,
                             "prepare_ms": 1000.0 * ph[0] / 3, "align_ms": 1000.0 * ph[1] / 3,
                             "points_per_cloud": int(np.mean(npts))}
        callers["note"] = ("rs_replay_app.cpp:229,246-251 per frame: RemoveNans, DownsampleVoxel "
                           "0.05 of both clouds (prepare_ms: with their unordered_map order, "
                           "k_umap_order), AlignIcp3d(curr_down, prev_down, 128) with its "
                           "index built per call (align_ms); host clouds (PCIe-inclusive), one "
                           "pair at a time")
        if not a.no_cpu and world == 1:
            callers["cpu_baseline"] = callers_cpu_baseline(raw, a.iters)
            for name in ("ref_sums", "fp64_sums"):
                callers[name]["speedup_vs_cpu"] = (callers["cpu_baseline"]["ms_per_pair"] /
                                                   callers[name]["ms_per_pair"])

    # ---- the tracker's GICP loop (rs_tracker.cpp:79-87; extra fields) ------------
    # per frame: DownsampleVoxel(curr, 0.1); ComputeAlignment(prev, curr, &T)
    # (16 rounds of exact NN + LM), host clouds, one pair at a time
    gicp = None
    if not a.no_gicp and not pyr:
        clouds = [A.DownsampleVoxel(driver.unproject(frames[pingpong(k, nfr)], K), 0.1)
                  for k in range(4)]
        T = np.eye(4, dtype=np.float32)
        A.ComputeAlignment(clouds[0], clouds[1], T)  # warm-up
        t3 = time.perf_counter()
        costs = []
        for k in range(1, 4):
            T = np.eye(4, dtype=np.float32)
            costs.append(A.ComputeAlignment(clouds[k - 1], clouds[k], T))
        dtg = (time.perf_counter() - t3) / 3
        gicp = {"ms_per_pair": 1000.0 * dtg, "pairs_per_s": 1.0 / dtg,
                "points_per_cloud": int(np.mean([len(c) for c in clouds])),
                "all_finite": bool(np.all(np.isfinite(costs))),
                "note": "rs_tracker.cpp loop: DownsampleVoxel(0.1) + GICP ComputeAlignment "
                        "(covariances k=32, 16 x {exact NN, fp64 LM <= 64 evaluations})"}

    # ---- roofline of the NN pass (k_icp_nn + k_icp_fb, one pair in flight) ----------
    nl1 = max(1, sr1["launches"])
    kern_us = [1000.0 * x / nl1 for x in sr1["iter_ms"]]  # nn | fb | rest, per iteration
    nn_us = kern_us[0] + kern_us[1]
    n_avg = st["n"] / max(1, npairs)
    m_avg = st["m"] / max(1, npairs)
    # a batched launch covers the batch's pairs: per-pair bytes x pairs per launch
    pairs_per_launch = sr1["batch_pairs"] / max(1, sr1["batches"]) if batched else 1.0
    # (point-to-plane also reads the target normals: 12 m more)
    alg_bytes = (p2point_alg_bytes(n_avg, m_avg) + (12 * m_avg if plane else 0)) * pairs_per_launch
    achieved = alg_bytes / (nn_us * 1e-6) / 1e9 if nn_us > 0 else 0.0
    # the committed PMC pass of this workload (scripts/gpu_evidence.sh,
    # gpu_configs.sh: the stream configs; the pyramid's levels and the
    # sharded pair have none)
    cfg_key = f"{a.workload}_{a.width}x{a.height}_{'p2plane' if plane else 'p2point_ref'}"
    traffic, traffic_src = (load_traffic(cfg_key) if a.workload == "stream" else
                            (None, "no PMC pass of this workload (its NN kernels run per level / "
                                   "per shard)"))
    if traffic is not None:
        traffic *= pairs_per_launch
    # the pyramid: every level's NN pass over its own kernel time (the levels
    # chained as the value leg runs them, one pair in flight)
    lv_roof = None
    if pyr:
        lv_roof = pyramid_level_roofline(a, d_depth, K, nfr, actx[0], pctx, opts_main, nk_main,
                                         pyr_iters)
        tb = sum(x["alg_bytes"] * x["iters"] for x in lv_roof)
        tt = sum(x["nn_us"] * x["iters"] for x in lv_roof)
        alg_bytes, nn_us = tb / max(1, sum(x["iters"] for x in lv_roof)), tt / max(1, sum(
            x["iters"] for x in lv_roof))
        achieved = tb / (tt * 1e-6) / 1e9 if tt > 0 else 0.0

    def sharded_extra() -> dict | None:
        """configs[3] beside the stream's line, on every rank: the 1M pair
        with its source sharded over ALL ranks of this run (RCCL over xGMI at
        N > 1), in the gated mode (RST_SUM_REF's relay), the fp64 mode and
        the north_star's point-to-plane split -- so a `--gpus N` run measures
        the collectives, not only replicas.  A watchdog bounds it: a leg
        that has not finished in --sharded-timeout s (a collective that never
        completes) ends the process with the stream's line printed."""
        if a.no_sharded or pyr or plane or a.workload != "stream":
            return None
        import threading
        state = {"done": False}

        def expire():
            if state["done"]:
                return
            if rank == 0 and "line" in state:
                line = dict(state["line"])
                line["sharded_1M"] = {"error": f"not finished in {a.sharded_timeout} s (watchdog)"}
                print(json.dumps(line), flush=True)
            os._exit(0)

        wd = threading.Timer(a.sharded_timeout, expire)
        wd.daemon = True
        state["timer"] = wd
        sw, sh_ = WORKLOADS["sharded"]
        Ks = driver.intrinsics(sw, sh_)
        sfr = render_frames(seed=0, n=2, K=Ks, stride=1)  # one pair, the same on every rank
        d_s = []
        for f in sfr:
            p = C.c_void_p()
            assert hip.hipMalloc(C.byref(p), C.c_size_t(2 * sw * sh_)) == 0
            assert hip.hipMemcpy(p, f.ctypes.data_as(C.c_void_p), C.c_size_t(2 * sw * sh_), 1) == 0
            d_s.append(p)
        return {"frames": d_s, "K": Ks, "size": (sw, sh_), "state": state}

    def sharded_run(prep) -> dict:
        st_ = prep["state"]
        st_["timer"].start()
        res = {"note": "configs[3]: one 1000x1000 pair (~1M points), the source sharded over "
                       f"all {world} rank(s) of this run, strong scaling; value = the pair's ICP "
                       "iterations/s (max over ranks); multi-rank RCCL unmeasured by the builder "
                       "(1-GPU boxes)", "n_ranks": world}
        try:
            for kind in ("ref", "fp64", "p2plane"):
                r = sharded_leg(kind, prep["size"][0], prep["size"][1], a.iters, a.sharded_steps, 2,
                                prep["frames"], local, rank, world, rdv, barrier, max_over_ranks,
                                hip, prep["K"])
                res[kind] = {k: r[k] for k in ("value", "ms_per_step", "iters_per_pair", "points",
                                               "shard_points", "pairs_ok", "nn_avg_us",
                                               "achieved_GBps", "accumulation", "exchange")}
        finally:
            st_["done"] = True
            st_["timer"].cancel()
            for p in prep["frames"]:
                hip.hipFree(p)
        return res

    sh_prep = sharded_extra()
    if rank != 0:
        if sh_prep is not None:
            sharded_run(sh_prep)
        rdv.close()
        return 0
    # the measured HBM ceiling on this box (stream copy, read + write bytes),
    # next to the spec peak the fraction is read against
    gb = C.c_double(0.0)
    cf = L.lib().rst_debug_stream_copy
    cf.restype, cf.argtypes = C.c_int, [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_double)]
    copy_gbps = gb.value if cf(actx[0].handle, 1 << 30, 5, C.byref(gb)) == 0 else None
    cpu = None
    if not a.no_cpu and world == 1:
        cpu = cpu_baseline(a.width, a.height, a.cpu_iters, pyr_iters if pyr else None)
    value = iters_all / dt
    out = {
        "metric": METRIC, "value": value, "unit": "ICP iterations/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "warmup_pairs": warm_steps * pps,
        "pairs": npairs, "pairs_per_step": pps,
        "ms_per_step": 1000.0 * dt / a.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded procedural RGB-D room, ray-cast u16 depth, 1 mm noise, "
                "~3% invalid)",
        "config": {"workload": (f"{a.width}x{a.height} synthetic RGB-D stream, per frame: "
                                f"{a.levels}-level pyramid (stride 2^l) unproject + index "
                                f"builds, coarse-to-fine P2POINT_REF ICP, iterations per "
                                f"level {pyr_iters} (finest first), pose chained on the device"
                                if pyr else
                                f"{a.width}x{a.height} synthetic RGB-D stream, per frame: "
                                f"unproject + image-grid normals (5x5 PCA) + index build + "
                                f"point-to-plane ICP to convergence (<= 30 iterations, 6x6 "
                                f"Gauss-Newton)"
                                if plane else
                                f"{a.width}x{a.height} synthetic RGB-D stream, per frame: "
                                f"unproject + index build + AlignIcp3d P2POINT_REF "
                                f"{a.iters} iters (reference loop)"),
                   "width": a.width, "height": a.height,
                   "mode": "P2PLANE" if plane else "P2POINT_REF",
                   "step": (f"one batch of {pps} consecutive frame pairs, aligned in lockstep "
                            f"(rst_icp_align_batch_async)" if batched else "one frame pair"),
                   "iters_per_pair": (round(st["iters"] / max(1, npairs), 2) if plane else
                                      sum(pyr_iters) if pyr else a.iters),
                   "iteration_unit": ("level-0 equivalents: a level-l iteration counts n_l / n_0"
                                      if pyr else "full-resolution ICP iteration"),
                   "points_per_frame": round(n_avg), "frames_cycled": nfr,
                   "accumulation": ("fp64 6x6 normal equations (point-to-plane; absent in the "
                                    "reference, SURVEY.md §8 a11)" if plane else
                                    "RST_SUM_REF: the reference's sequential fp32 sums, "
                                    "bit-exact (the drop-in default; within the 1e-4 gate)"
                                    if main_ref else
                                    "RST_SUM_FP64: fp64 partial sums (not the drop-in "
                                    "default; outside the 1e-4 gate of the reference's fp32 "
                                    "sums, see ref_sums)"),
                   "parallelism": f"replica{world}",
                   "pairs_in_flight_per_gpu": len(actx) * (a.batch if batched else 1),
                   "pairs_per_batch": a.batch if batched else 1,
                   "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                   "hipgraph": bool(a.graphs)},
        "frames_per_s": frames_all / dt,
        "pairs_ok": st["ok"],
        **({"iterations_all_levels_per_s": iters_raw / dt} if pyr else {}),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "stream_copy_GBps": copy_gbps,
                     "kernel": ("k_icp_nn_b+k_icp_fb_b (one ICP iteration's NN pass of a batch "
                                f"of {pairs_per_launch:g} pairs: certificate stream + compacted "
                                "searches)" if batched else
                                "k_icp_nn+k_icp_fb (one ICP iteration's NN pass: certificate "
                                "stream + compacted searches)"),
                     "pairs_per_launch": pairs_per_launch,
                     **({"levels": lv_roof,
                         "levels_note": "each level's NN-pass bytes over its own kernel time; "
                                        "achieved / frac above: all levels' bytes x iterations "
                                        "over their kernel time x iterations"} if lv_roof else {}),
                     "avg_us": nn_us, "alg_bytes_per_launch": alg_bytes,
                     "kernels_avg_us": {"k_icp_nn": kern_us[0], "k_icp_fb": kern_us[1],
                                        "rest_of_iteration": kern_us[2]},
                     "timing": (f"HIP events around every iteration's kernels, one "
                                f"{'batch' if batched else 'pair'} in flight, "
                                f"{sr1['batch_pairs'] if batched else a.roof_steps} frame pairs "
                                f"({sr1['launches']} iterations)"),
                     "traffic_source": traffic_src},
        "cpu_baseline": cpu,
    }
    if pl is not None:
        out["p2plane"] = pl
    if refs is not None:
        out["fp64_sums" if main_ref else "ref_sums"] = refs
    if host is not None:
        out["host_api"] = host
    if callers is not None:
        out["callers_workload"] = callers
    if gicp is not None:
        out["gicp"] = gicp
    if cpu is not None:
        out["speedup_vs_cpu_baseline"] = value / cpu["value"]
    if sh_prep is not None:
        sh_prep["state"]["line"] = out  # (printed by the watchdog if the leg never finishes)
        out["sharded_1M"] = sharded_run(sh_prep)
    print(json.dumps(out))
    rdv.close()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
