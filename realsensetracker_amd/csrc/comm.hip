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
// [off_r, off_r + n_r).  Each iteration every rank all-gathers the
// correspondences (q, d2 per source point, 16 B) into the whole source's
// order -- one grouped set of broadcasts, ranks' counts may differ -- and
// walks the global chains redundantly (seqsum.hip), so every rank holds the
// same bit-exact dst_mean and cost; the covariance stays a sharded fp64
// partial sum (9 doubles all-reduced).
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
  int64_t layout_local = -1, layout_total = -1;
  std::vector<int64_t> counts, offsets;
  int64_t* d_cnt = nullptr;  // device scratch of the count all-gather
};

namespace rst {

int comm_allreduce_sum_f64(rst_comm* comm, double* d_buf, size_t count, hipStream_t stream) {
  if (!comm || !comm->comm) return RST_E_ARG;
  if (ncclAllReduce(d_buf, d_buf, count, ncclFloat64, ncclSum, comm->comm, stream) != ncclSuccess)
    return RST_E_COMM;
  return RST_OK;
}

int comm_size(const rst_comm* comm) { return comm ? comm->nranks : 1; }

// Every rank's shard size.  The exchange (one all-gather of one int64 per
// rank and a host synchronisation) runs on the first align of a
// communicator, whenever the caller passes no n_total, and whenever this
// rank's n_local or the caller's n_total differ from the cached layout's
// (a shard-size change must therefore reach every rank in the same align,
// or the caller passes n_total = 0 on every rank); a given n_total is
// checked against the exchanged counts, so a wrong or rank-dependent value
// fails with RST_E_ARG instead of skewing the means.
int comm_shard_layout(rst_comm* comm, int64_t n_local, int64_t n_total_hint, hipStream_t st,
                      int64_t* n_total, int64_t* offset, const std::vector<int64_t>** counts) {
  if (!comm || !comm->comm) return RST_E_ARG;
  const bool cached = comm->have_layout && n_total_hint > 0 && n_local == comm->layout_local &&
                      n_total_hint == comm->layout_total;
  if (!cached) {
    const int R = comm->nranks;
    if (!comm->d_cnt && hipMalloc(&comm->d_cnt, sizeof(int64_t) * (R + 1)) != hipSuccess)
      return RST_E_NOMEM;
    RST_HIP(hipMemcpyAsync(comm->d_cnt + R, &n_local, sizeof(int64_t), hipMemcpyHostToDevice, st));
    if (ncclAllGather(comm->d_cnt + R, comm->d_cnt, 1, ncclInt64, comm->comm, st) != ncclSuccess)
      return RST_E_COMM;
    std::vector<int64_t> c(R);
    RST_HIP(hipMemcpyAsync(c.data(), comm->d_cnt, sizeof(int64_t) * R, hipMemcpyDeviceToHost, st));
    RST_HIP(hipStreamSynchronize(st));
    std::vector<int64_t> o(R);
    int64_t tot = 0;
    for (int r = 0; r < R; ++r) {
      if (c[r] < 0) return RST_E_ARG;
      o[r] = tot;
      tot += c[r];
    }
    if (c[comm->rank] != n_local) return RST_E_ARG;
    comm->counts = c;
    comm->offsets = o;
    comm->layout_local = n_local;
    comm->layout_total = tot;
    comm->have_layout = true;
  }
  if (n_total_hint > 0 && n_total_hint != comm->layout_total) return RST_E_ARG;
  *n_total = comm->layout_total;
  *offset = comm->offsets[comm->rank];
  if (counts) *counts = &comm->counts;
  return RST_OK;
}

// buf[off_r, off_r + n_r) of rank r to every rank (in place; counts may
// differ): grouped broadcasts, one per non-empty shard
int comm_allgatherv_f4(rst_comm* comm, float4* buf, hipStream_t st) {
  if (!comm || !comm->comm || !comm->have_layout) return RST_E_ARG;
  if (ncclGroupStart() != ncclSuccess) return RST_E_COMM;
  ncclResult_t e = ncclSuccess;
  for (int r = 0; r < comm->nranks && e == ncclSuccess; ++r) {
    const size_t cnt = (size_t)comm->counts[r] * 4;
    if (cnt == 0) continue;
    float* p = reinterpret_cast<float*>(buf + comm->offsets[r]);
    e = ncclBroadcast(p, p, cnt, ncclFloat32, r, comm->comm, st);
  }
  if (ncclGroupEnd() != ncclSuccess || e != ncclSuccess) return RST_E_COMM;
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
  if (comm->d_cnt) {
    (void)hipSetDevice(comm->device);
    (void)hipFree(comm->d_cnt);
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
