// comm.hip -- multi-GPU ICP over RCCL (xGMI).
//
// The reference has no distribution at all.  The path shards
// by source points: every rank holds the full target index (built
// redundantly from the same frame) and a contiguous shard of the source; per
// iteration each rank reduces its fp64 partial sums to one row
// (16 P2POINT_REF / 30 P2PLANE doubles, <= 240 B) and ONE ncclAllReduce
// makes the normal equations global; every rank then solves the same pose,
// so no broadcast follows.  The message is latency-bound, not link-bound.
//
// RST_SUM_REF (the reference's sequential fp32 sums) shards too: the shards
// are contiguous stretches of the reference's source order, rank r holding
// [off_r, off_r + n_r).  Each iteration every rank maps the chains of its own
// stretch and the chains' values travel rank to rank (comm_relay_seqsum:
// < 1 KB per iteration), so every rank holds the same bit-exact dst_mean and
// cost; the covariance stays a sharded fp64 partial sum (9 doubles
// all-reduced).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "rst_internal.hpp"

struct rst_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1;
  int rank = 0;
  int device = 0;
  // the shard layout of the last count exchange (rst::comm_shard_layout)
  bool have_layout = false;
  int64_t layout_total = -1;
  std::vector<int64_t> counts, offsets;
  int64_t* d_cnt = nullptr;     // device scratch of the count all-gather [R + 1]
  int64_t* d_layout = nullptr;  // the exchanged counts on the device [R]
  double* d_relay = nullptr;    // comm_relay_seqsum's exchange buffers
  int32_t* d_guards = nullptr;  // comm_agree_guard's all-gather [R + 1]
};

namespace rst {

int comm_allreduce_sum_f64(rst_comm* comm, double* d_buf, size_t count, hipStream_t stream) {
  if (!comm || !comm->comm) return RST_E_ARG;
  if (ncclAllReduce(d_buf, d_buf, count, ncclFloat64, ncclSum, comm->comm, stream) != ncclSuccess)
    return RST_E_COMM;
  return RST_OK;
}

int comm_size(const rst_comm* comm) { return comm ? comm->nranks : 1; }

namespace {
__global__ void k_put_i64(int64_t* __restrict__ p, int64_t v) {
  if (threadIdx.x == 0) *p = v;
}
// this align's all-gathered counts against the cached layout: a rank whose
// shard size changed without an n_total change shows up in every rank's
// copy of the gathered counts, so every rank flags the same align
__global__ void k_layout_check(const int64_t* __restrict__ got, const int64_t* __restrict__ want, int R,
                               int32_t* __restrict__ guard) {
  bool bad = false;
  for (int r = threadIdx.x; r < R; r += blockDim.x) bad = bad || got[r] != want[r];
  if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(guard, kGuardLayout);
}
}  // namespace

// Every rank's shard size.  Whether the sizes are exchanged (one all-gather
// of an int64 per rank and a host synchronisation) depends only on values
// every rank holds alike -- the communicator's first align, a caller's
// n_total of 0, or an n_total other than the cached layout's -- so the ranks
// always issue the same collectives (the caller passes the same n_total on
// every rank: include/rst_align.h).  An exchange whose total differs from a
// given n_total fails with RST_E_ARG on every rank (they all see the same
// counts) before any further collective.  With the cached layout, every
// align still all-gathers the ranks' counts (no host wait) and
// comm_layout_check compares them with the cache on the device: a shard
// size changed at an unchanged n_total fails that align on every rank at
// icp_finish (RST_E_ARG).  *n_eff is the source count this rank runs with
// (0 when its size left the layout), so a stale layout never moves a kernel
// out of its buffers.
int comm_shard_layout(rst_comm* comm, int64_t n_local, int64_t n_total_hint, hipStream_t st,
                      int64_t* n_total, int64_t* offset, int64_t* n_eff,
                      const std::vector<int64_t>** counts) {
  if (!comm || !comm->comm) return RST_E_ARG;
  const int R = comm->nranks;
  if (!comm->d_cnt) {
    if (hipMalloc(&comm->d_cnt, sizeof(int64_t) * (2 * R + 1)) != hipSuccess) return RST_E_NOMEM;
    comm->d_layout = comm->d_cnt + R + 1;
  }
  const bool exchange = !comm->have_layout || n_total_hint <= 0 || n_total_hint != comm->layout_total;
  k_put_i64<<<1, 64, 0, st>>>(comm->d_cnt + R, n_local);
  RST_HIP(hipGetLastError());
  if (ncclAllGather(comm->d_cnt + R, comm->d_cnt, 1, ncclInt64, comm->comm, st) != ncclSuccess)
    return RST_E_COMM;
  if (exchange) {
    std::vector<int64_t> c(R);
    RST_HIP(hipMemcpyAsync(c.data(), comm->d_cnt, sizeof(int64_t) * R, hipMemcpyDeviceToHost, st));
    RST_HIP(hipStreamSynchronize(st));
    std::vector<int64_t> o(R);
    int64_t tot = 0;
    bool neg = false;
    for (int r = 0; r < R; ++r) {
      neg = neg || c[r] < 0;
      o[r] = tot;
      tot += c[r];
    }
    comm->have_layout = false;
    if (neg) return RST_E_ARG;  // (every rank sees the same counts)
    comm->counts = c;
    comm->offsets = o;
    comm->layout_total = tot;
    comm->have_layout = true;
    RST_HIP(hipMemcpyAsync(comm->d_layout, comm->counts.data(), sizeof(int64_t) * R, hipMemcpyHostToDevice,
                           st));
    RST_HIP(hipStreamSynchronize(st));
  }
  if (n_total_hint > 0 && n_total_hint != comm->layout_total) return RST_E_ARG;
  *n_total = comm->layout_total;
  *offset = comm->offsets[comm->rank];
  // (a rank whose size left the cached layout runs no points: its searches
  // scatter to original indices up to its own size, which the layout would
  // not hold; the align is flagged on every rank by comm_layout_check)
  *n_eff = n_local == comm->counts[comm->rank] ? n_local : 0;
  if (counts) *counts = &comm->counts;
  return RST_OK;
}

int comm_layout_check(rst_comm* comm, hipStream_t st, int32_t* d_guard) {
  if (!comm || !comm->d_cnt) return RST_E_ARG;
  k_layout_check<<<1, 64, 0, st>>>(comm->d_cnt, comm->d_layout, comm->nranks, d_guard);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

namespace {
__global__ void k_guard_copy(const int32_t* __restrict__ guard, int32_t* __restrict__ out) {
  if (threadIdx.x == 0) *out = *guard;
}
__global__ void k_guard_or(const int32_t* __restrict__ all, int R, int32_t* __restrict__ guard) {
  if (threadIdx.x != 0) return;
  int32_t g = *guard;
  for (int r = 0; r < R; ++r) g |= all[r];
  *guard = g;
}
}  // namespace

int comm_agree_guard(rst_comm* comm, hipStream_t st, int32_t* d_guard) {
  if (!comm || !comm->comm || !d_guard) return RST_E_ARG;
  const int R = comm->nranks;
  if (!comm->d_guards && hipMalloc(&comm->d_guards, sizeof(int32_t) * (R + 1)) != hipSuccess) return RST_E_NOMEM;
  k_guard_copy<<<1, 64, 0, st>>>(d_guard, comm->d_guards + R);
  RST_HIP(hipGetLastError());
  if (ncclAllGather(comm->d_guards + R, comm->d_guards, 1, ncclInt32, comm->comm, st) != ncclSuccess)
    return RST_E_COMM;
  k_guard_or<<<1, 64, 0, st>>>(comm->d_guards, R, d_guard);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

namespace {
// the relay's guesses: the fp64 prefix of the ranks before this one (their
// chain totals), plus the drift the previous iteration's true start showed
__global__ void k_relay_p0(const double* __restrict__ tots, int R, int rank, const double* __restrict__ drift,
                           double* __restrict__ p0raw, double* __restrict__ p0) {
  const int c = threadIdx.x;
  if (c >= 4) return;
  double s = 0.0;
  for (int r = 0; r < rank && r < R; ++r) s += tots[r * 4 + c];
  p0raw[c] = s;
  p0[c] = s + (drift ? drift[c] : 0.0);
}
// the float chain's value at the stretch start against the fp64 prefix there
// (the next iteration's guesses start from it; the chains move little)
__global__ void k_relay_drift(const float* __restrict__ s_in, const double* __restrict__ p0raw,
                              double* __restrict__ drift) {
  const int c = threadIdx.x;
  if (c >= 4) return;
  const float v = s_in[c];
  drift[c] = isfinite(v) && isfinite(p0raw[c]) ? (double)v - p0raw[c] : 0.0;
}
}  // namespace

// The reference's sequential fp32 sums over the ranks' stretches, in order
// (align_icp.cpp:113,120; point_cloud_utils.cpp:94-96), without moving the
// stretches: every rank maps its own stretch (seqsum.hip) with the fp64
// prefix of the ranks before it as the guesses' offset (one all-gather of
// the ranks' fp64 totals, 32 B each), rank r - 1 hands rank r the chains'
// value at the stretch start (ncclRecv / ncclSend, 16 B), rank r walks its
// stretch from it, and the last rank broadcasts the sums (16 B).  The walks
// follow one another -- a sequential sum has no other decomposition -- but
// each covers n / R elements, with its own descents, and the maps, the
// bulk of the work, shrink by R and run on every rank at once (enqueued
// ahead of the receive: only the walk waits on the rank before).  d_out: 4 floats on every rank; d_drift (4
// doubles, zero at an align's start, or null) carries the start's drift
// from one iteration to the next.
int comm_relay_seqsum(rst_comm* comm, const float4* d_x, int64_t n_local, int nch, void* sqws,
                      float* d_out, hipStream_t st, double* d_drift, int* d_stats, int iter, int* d_guard) {
  if (!comm || !comm->comm || nch < 1 || nch > 4) return RST_E_ARG;
  const int R = comm->nranks, rank = comm->rank;
  if (!comm->d_relay) {
    const size_t b = sizeof(double) * (4 + 4 * (size_t)R + 8) + sizeof(float) * 4;
    if (hipMalloc(&comm->d_relay, b) != hipSuccess) return RST_E_NOMEM;
  }
  double* tot4 = comm->d_relay;
  double* tots = tot4 + 4;
  double* p0raw = tots + 4 * R;
  double* p0 = p0raw + 4;
  float* s_in = (float*)(p0 + 4);
  RST_CHECK(seqsum_totals(d_x, n_local, nch, sqws, tot4, st, iter));
  if (ncclAllGather(tot4, tots, 4, ncclFloat64, comm->comm, st) != ncclSuccess) return RST_E_COMM;
  k_relay_p0<<<1, 64, 0, st>>>(tots, R, rank, d_drift, p0raw, p0);
  RST_HIP(hipGetLastError());
  const SqStretch sx{p0, s_in, true};
  // the maps need only the guesses (p0): enqueued before the receive, so rank
  // r maps its stretch while the ranks before it walk theirs; only the walk
  // (which alone reads s_in) waits for rank r - 1's chain values
  const bool split = n_local > 0;
  if (split) RST_CHECK(seqsum_enqueue(d_x, n_local, nch, sqws, d_out, st, d_stats, 3, iter, false, &sx, nullptr, d_guard));
  if (rank > 0) {
    if (ncclRecv(s_in, 4, ncclFloat32, rank - 1, comm->comm, st) != ncclSuccess) return RST_E_COMM;
  } else {
    RST_HIP(hipMemsetAsync(s_in, 0, sizeof(float) * 4, st));
  }
  RST_CHECK(seqsum_enqueue(d_x, n_local, nch, sqws, d_out, st, d_stats, split ? 4 : 7, iter, false, &sx, nullptr,
                           d_guard));
  if (rank + 1 < R && ncclSend(d_out, 4, ncclFloat32, rank + 1, comm->comm, st) != ncclSuccess)
    return RST_E_COMM;
  if (ncclBroadcast(d_out, d_out, 4, ncclFloat32, R - 1, comm->comm, st) != ncclSuccess) return RST_E_COMM;
  if (d_drift) {
    k_relay_drift<<<1, 64, 0, st>>>(s_in, p0raw, d_drift);
    RST_HIP(hipGetLastError());
  }
  return RST_OK;
}

}  // namespace rst

using namespace rst;

extern "C" {

int rst_comm_get_unique_id(char id_out[RST_COMM_ID_BYTES]) {
  if (!id_out) return RST_E_ARG;
  static_assert(sizeof(ncclUniqueId) <= RST_COMM_ID_BYTES, "id size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return RST_E_COMM;
  memset(id_out, 0, RST_COMM_ID_BYTES);
  memcpy(id_out, &id, sizeof(id));
  return RST_OK;
}

int rst_comm_create(rst_ctx* ctx, const char id[RST_COMM_ID_BYTES], int nranks, int rank,
                    rst_comm** out) {
  if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  rst_comm* c = new rst_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = ctx->device;
  if (ncclCommInitRank(&c->comm, nranks, uid, rank) != ncclSuccess) {
    delete c;
    return RST_E_COMM;
  }
  *out = c;
  return RST_OK;
}

int rst_comm_destroy(rst_comm* comm) {
  if (!comm) return RST_OK;
  if (comm->comm) ncclCommDestroy(comm->comm);
  if (comm->d_cnt || comm->d_relay || comm->d_guards) {
    (void)hipSetDevice(comm->device);
    if (comm->d_cnt) (void)hipFree(comm->d_cnt);
    if (comm->d_relay) (void)hipFree(comm->d_relay);
    if (comm->d_guards) (void)hipFree(comm->d_guards);
  }
  delete comm;
  return RST_OK;
}

int rst_icp_align_sharded_device(rst_ctx* ctx, rst_comm* comm, const float* d_src_shard,
                                 int64_t n_shard, const rst_target* tgt,
                                 const rst_icp_opts* opts, float pose_inout[16],
                                 float* mean_cost) {
  if (!ctx || !comm || !tgt || !pose_inout || n_shard < 0 || (n_shard > 0 && !d_src_shard))
    return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  rst_target* s = nullptr;
  RST_CHECK(target_build_device(ctx, d_src_shard, n_shard, false, &s));
  int r = icp_align_prepared(ctx, s, tgt, opts, pose_inout, mean_cost, nullptr, comm);
  rst_target_free(s);
  return r;
}

int rst_icp_align_sharded_prepared(rst_ctx* ctx, rst_comm* comm, const rst_target* src_shard,
                                   const rst_target* tgt, const rst_icp_opts* opts,
                                   float pose_inout[16], float* mean_cost) {
  if (!ctx || !comm || !src_shard || !tgt || !pose_inout) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return icp_align_prepared(ctx, src_shard, tgt, opts, pose_inout, mean_cost, nullptr, comm);
}

}  // extern "C"
