// comm.hip -- multi-GPU ICP over RCCL (xGMI).
//
// The reference has no distribution at all.  The path shards
// by source points: every rank holds the full target index (built
// redundantly from the same frame) and a contiguous shard of the source; per
// iteration each rank reduces its fp64 partial sums to one row
// (16 P2POINT_REF / 30 P2PLANE doubles, <= 240 B) and ONE ncclAllReduce
// makes the normal equations global; every rank then solves the same pose,
// so no broadcast follows.  The message is latency-bound, not link-bound.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "rst_internal.hpp"

struct rst_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1;
  int rank = 0;
  int device = 0;
};

namespace rst {

int comm_allreduce_sum_f64(rst_comm* comm, double* d_buf, size_t count, hipStream_t stream) {
  if (!comm || !comm->comm) return RST_E_ARG;
  if (ncclAllReduce(d_buf, d_buf, count, ncclFloat64, ncclSum, comm->comm, stream) != ncclSuccess)
    return RST_E_COMM;
  return RST_OK;
}

int comm_size(const rst_comm* comm) { return comm ? comm->nranks : 1; }

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
  // a sequential sum over the whole source has no shard decomposition: the
  // sharded loop always reduces fp64 partial sums (rst_align.h sum_mode)
  rst_icp_opts o;
  if (opts)
    o = *opts;
  else
    rst_icp_opts_default(&o);
  o.sum_mode = RST_SUM_FP64;
  rst_target* s = nullptr;
  RST_CHECK(target_build_device(ctx, d_src_shard, n_shard, false, &s));
  int r = icp_align_prepared(ctx, s, tgt, &o, pose_inout, mean_cost, nullptr, comm);
  rst_target_free(s);
  return r;
}

int rst_icp_align_sharded_prepared(rst_ctx* ctx, rst_comm* comm, const rst_target* src_shard,
                                   const rst_target* tgt, const rst_icp_opts* opts,
                                   float pose_inout[16], float* mean_cost) {
  if (!ctx || !comm || !src_shard || !tgt || !pose_inout) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  rst_icp_opts o;
  if (opts)
    o = *opts;
  else
    rst_icp_opts_default(&o);
  o.sum_mode = RST_SUM_FP64;
  return icp_align_prepared(ctx, src_shard, tgt, &o, pose_inout, mean_cost, nullptr, comm);
}

}  // extern "C"
