// rst_internal.hpp -- host-side objects of the MI355X ICP library.
//
// One rst_ctx = one GPU + one HIP stream + grow-only workspaces.  One
// rst_target = one prepared cloud resident in HBM: Morton-sorted points
// (float4 x,y,z,orig-index-bits), the implicit BVH over them, optional
// normals.  See DESIGN.md "Data layout in HBM".
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "rst_align.h"
#include "rst_bvh.hpp"

namespace rst {

// ---- error plumbing -------------------------------------------------------
#define RST_HIP(call)                                                     \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess) {                                               \
      rst::set_last_error(e_, #call, __FILE__, __LINE__);                 \
      return RST_E_HIP;                                                   \
    }                                                                     \
  } while (0)

#define RST_CHECK(expr)            \
  do {                             \
    int s_ = (expr);               \
    if (s_ < 0) return s_;         \
  } while (0)

void set_last_error(hipError_t e, const char* what, const char* file,
                    int line);

// BVH geometry: rst_bvh.hpp.

// ---- device-resident state of one ICP solve --------------------------------
// Written only by the single-block solve kernels, read (uniformly) by the
// per-point kernels.  Plain POD; lives in the context's workspace.
constexpr int kQTrace = 256;
#ifndef RST_TIMELINE
#define RST_TIMELINE 0  // diagnostics build: device-side kernel timeline of the ICP loop
#endif
// the loop's kernels in the timeline: nn, fb, sq_tot, sq_front, sq_build,
// sq_walk, cov_ref, reduce_solve
constexpr int kTlKernels = 8;
#if RST_TIMELINE && defined(__HIPCC__)
// (light: the start from block 0's first wave, the end from the first wave of
// the grid's last four blocks -- dispatched last, done about last; one
// atomic per wave on one address serialised the kernels it measured)
struct TlGuard {
  unsigned long long* p;
  bool first, last;
  __device__ TlGuard(unsigned long long* base, int it, int kid)
      : p(base && it >= 0 && it < kQTrace ? base + ((size_t)it * kTlKernels + kid) * 2 : nullptr),
        first(blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0),
        last(blockIdx.x + 4 >= gridDim.x && threadIdx.x == 0) {
    if (p && first) atomicMin(p, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
  __device__ ~TlGuard() {
    if (p && last) atomicMax(p + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
};
#define RST_TL(base, it, kid) rst::TlGuard rst_tl_guard_((base), (it), (kid))
#else
#define RST_TL(base, it, kid) (void)0
#endif
// IcpCore::guard bit of a shard layout that changed at an unchanged n_total
constexpr int32_t kGuardLayout = 1 << 16;
// ... and of a sequential-sum table bound check that tripped (seqsum.hip
// err bits above kGuardSeqsumShift): the sums are not trusted
constexpr int32_t kGuardSeqsum = 1 << 17, kGuardSeqsumShift = 20;

// The part of the state the solve reads and writes: copied to registers at
// the start of the solve kernel (its loads overlap the slab reduction) and
// written back at the end.
struct IcpCore {
  float R[9];        // current pose, column-major (what the points see)
  float t[3];
  float smean[3];    // source centroid (P2POINT_REF)
  float mu;          // annealing parameter for the next iteration
  int32_t iter;      // iterations completed
  int32_t done;      // P2PLANE converged / failed flag
  float last_cost;   // sum d2 of the last iteration (as float)
  float pad0;
  double Rd[9];      // P2PLANE high-precision pose
  double td[3];
  double last_xi;    // |xi| of the last P2PLANE step
  double last_cnt;   // accepted correspondences of the last step
  double last_d2;    // sum d2 of the last step
  int32_t fail;      // P2PLANE: singular system / too few points
  int32_t fb_e;      // fallback-queue entries of the current iteration
  float seq[4];      // RST_SUM_REF: this iteration's sequential fp32 sums
                     // (sum dst[nbr_i] xyz, cost), align_icp.cpp:113,120
  int32_t guard;     // bit mask of index guards that tripped (0: none; diagnostics);
                     // kGuardLayout: a sharded align's shard sizes changed at an
                     // unchanged n_total (comm.hip)
  int32_t pad1;
};

struct IcpState : IcpCore {
  float in_pose[12];      // the solve's initial pose (R col-major, t): a pyramid
                          // level that fails chains this on (host semantics)
  int32_t qlen[kQTrace];  // fallback-queue length per iteration (diagnostics)
  int32_t path[kQTrace][4];  // per-iteration diagnostics (rst_debug_queue_trace)
  int32_t diag[kQTrace][4];  // RST_DIAG builds: far queue, ball chunks, ball aborts, deep searches
  float seqtr[kQTrace][4];   // RST_SUM_REF: each iteration's sequential sums (sum q xyz, cost;
                             // the cost every iteration only under rst_debug_enable_seq_trace)
#if RST_TIMELINE
  // diagnostics build: per iteration and loop kernel, the earliest wave start
  // and the latest wave end (100 MHz real-time clock; rst_debug_timeline)
  unsigned long long tl[kQTrace][kTlKernels][2];
#endif
};

struct IcpParams {
  int64_t n;           // total source points (all shards)
  int32_t anneal_every;
  float anneal_div;
  float p2plane_eps;
  float p2plane_mu;
  float p2plane_max_d2;
  int32_t max_iter;
  int32_t lane_min;    // fallback queue length from which it runs one lane per query
  int32_t sum_mode;    // rst_sum_mode
};

}  // namespace rst

// ---- public opaque objects ------------------------------------------------
struct rst_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // workspaces (grow-only)
  void* ws = nullptr;
  size_t ws_bytes = 0;
  void* pinned = nullptr;     // host staging: two halves of kStageChunk bytes
  size_t pinned_bytes = 0;
  hipEvent_t stage_ev[2] = {nullptr, nullptr};  // the last copy through each half
  rst::IcpState* d_state = nullptr;
  rst::IcpState* h_state = nullptr;   // pinned mirror
  double* d_slab = nullptr;           // per-block partial sums
  size_t slab_bytes = 0;
  // timing of the dominant per-iteration kernel
  bool timing = false;
  int timing_stride = 1;              // time every timing_stride-th iteration
  std::vector<hipEvent_t> ev;
  float last_kernel_ms = 0.f;
  float last_iter_ms[3] = {0.f, 0.f, 0.f};  // k_icp_nn | k_icp_fb | the rest of the iteration
  int32_t last_kernel_launches = 0;
  int32_t last_iters = 0;  // iterations the last finished align ran (rst_ctx_last_iterations)
  // hipGraph replay of the ICP iteration loop (rst_ctx_enable_graphs):
  // (pyramid level, iterations, P2PLANE, RST_SUM_REF) -> executable graph,
  // updated in place per align
  bool graphs = false;
  bool seq_trace = false;  // RST_SUM_REF: walk the cost chain every iteration (diagnostics)
  int32_t* d_sqstats = nullptr;  // with seq_trace: the walks' statistics, 64 int32 per iteration
  std::map<std::tuple<int, int, int, int>, hipGraphExec_t> gexec;
  // device memory of freed targets, kept for the next build (hipFree
  // synchronises the whole device, which would stall every stream of a
  // pipelined frame loop): size class -> blocks
  std::multimap<size_t, void*> pool;
  size_t pool_bytes = 0;
  std::vector<rst_target*> live;  // targets built on this context
  // guards pool / pool_bytes / live: a target may be freed on another host
  // thread than the one building the next (a frame-preparation thread)
  std::mutex pool_mu;
  // the align enqueued by icp_launch and not yet collected by icp_finish
  struct Pending {
    bool early_false = false;
    bool active = false;
    bool p2plane = false;
    bool timing = false;
    bool pyramid = false;  // rst_icp_align_pyramid_async: a failed level 0 hands back its input
    int32_t max_iter = 0;
    int64_t n_total = 0;
  } pend;
  // a batch of frame pairs aligned in lockstep (rst_icp_align_batch_async):
  // one IcpState per pair, device and pinned host mirrors, grown on demand
  rst::IcpState* d_bstate = nullptr;
  rst::IcpState* h_bstate = nullptr;
  int32_t bcap = 0;
  struct PendingBatch {
    bool active = false;
    bool p2plane = false;
    bool timing = false;
    int32_t nb = 0;        // pairs in the call
    int32_t max_iter = 0;
    std::vector<int32_t> slot;     // per pair: its state slot, -1 = the reference's early false
    std::vector<int64_t> n_total;  // per pair
  } bpend;
};

struct rst_target {
  rst_ctx* ctx = nullptr;
  int64_t m = 0;
  int32_t nleaves = 0;
  int32_t lg = 0;               // nleaves = 1 << lg
  float4* pts = nullptr;        // [m] Morton-sorted (x,y,z,orig idx bits)
  float4* nodes = nullptr;      // [2 * 2*nleaves]
  int32_t* lstart = nullptr;    // [nleaves + 1] leaf ranges (rst_bvh.hpp)
  int32_t* pleaf = nullptr;     // [m] leaf of each sorted point
  int32_t* inv = nullptr;       // [m] original index -> sorted position
  uint32_t* codes = nullptr;    // [m] sorted Morton codes, then 6 floats: their box
  float4* adj = nullptr;        // [nleaves * kAdjK * 2] leaf adjacency (rst_bvh.hpp)
  float* reach = nullptr;       // [nleaves]
  float4* adj2 = nullptr;       // the same over the nodes of 8 leaves
  float* reach2 = nullptr;
  float4* adj3 = nullptr;       // ... and over the nodes of 64 leaves
  float* reach3 = nullptr;
  float4* nrm = nullptr;        // [m] normals in sorted order (optional)
  rst::PixView pix = {};        // pixel grid -> sorted position (frames from depth only)
  float bbox[6] = {0, 0, 0, 0, 0, 0};
  int32_t pos0 = 0;             // sorted position of original point 0
  bool has_bvh = false;
  std::vector<std::pair<void*, size_t>> allocs;  // every device block (size class)
};

namespace rst {

// device memory through the context's pool (capi.hip): blocks are rounded
// to a size class (1/8 of a power of two), reused first-fit by class
int ctx_alloc(rst_ctx* ctx, size_t bytes, void** out, size_t* class_bytes);
void ctx_release(rst_ctx* ctx, void* p, size_t class_bytes);
// a target-owned block (freed with the target)
int target_alloc(rst_target* t, size_t bytes, void** out);

// workspace helpers (implemented in capi.hip)
int ctx_workspace(rst_ctx* ctx, size_t bytes, void** out);
// host <-> device copies through the context's pinned staging buffer, in
// chunks of at most kStageChunk bytes through two alternating halves (one
// half's DMA in flight while the other is filled): the pinned memory stays
// 2 x kStageChunk however large the copy.  h2d returns with the copies
// enqueued on the context's stream (h may be reused at once); d2h returns
// with h written.
constexpr size_t kStageChunk = (size_t)8 << 20;
// a separate small pinned area past the halves (device -> host flags)
constexpr size_t kPinnedSmall = 4096;
int ctx_pinned_small(rst_ctx* ctx, size_t bytes, void** out);
int stage_h2d(rst_ctx* ctx, void* d, const void* h, size_t bytes);
int stage_d2h(rst_ctx* ctx, void* h, const void* d, size_t bytes);
int ctx_slab(rst_ctx* ctx, size_t bytes, double** out);

// target build (build.hip)
int target_build_device(rst_ctx* ctx, const float* d_xyz, int64_t m,
                        bool with_bvh, rst_target** out);
size_t target_index_bytes(const rst_target* t);
BvhView view_of(const rst_target* t);
AdjView adj_of(const rst_target* t);

// NN queries (query.hip)
int query_nn_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q,
                    int64_t nq, int32_t* d_idx, float* d_d2);
int query_nn_warm_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q, int64_t nq,
                         const int32_t* d_warm, int32_t* d_idx, float* d_d2,
                         int* d_stats = nullptr);
int query_nn_fallback_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q, int64_t nq,
                             const int32_t* d_warm, int mode, int32_t* d_idx, float* d_d2,
                             int32_t* d_path);
int query_knn_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q,
                     int64_t nq, int k, int32_t* d_idx, float* d_d2);
int compute_normals(rst_ctx* ctx, rst_target* tgt, int k, const float vp[3]);
// image-grid normals over a (2r+1)^2 pixel window (frame targets only)
int compute_grid_normals(rst_ctx* ctx, rst_target* tgt, int r, const float vp[3]);

// ICP (icp.hip)
int icp_launch(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
               const rst_icp_opts* opts, const float pose_in[16], rst_comm* comm,
               bool chain = false, int level = 0);
// diagnostics (rst_debug.h): one iteration's partial sums; the solve step
int icp_debug_partials(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
                       const rst_icp_opts* opts, const float pose[16], float mu,
                       const float smean[3], int32_t iter, double* out, int32_t* nv);
int icp_debug_solve(rst_ctx* ctx, const rst_icp_opts* opts, int64_t n_total,
                    const double* totals, const float smean[3], float pose_inout[16],
                    float* mu_inout, int32_t* iter_inout);
int icp_finish(rst_ctx* ctx, float pose_inout[16], float* mean_cost, int32_t* iters_run);
// a batch of nb independent pairs in lockstep: one launch per loop kernel for
// the whole batch (pairs with the reference's early false are left out and
// reported so by icp_finish_batch); then per pair the same results as
// icp_finish (status RST_OK / RST_FALSE per pair)
int icp_launch_batch(rst_ctx* ctx, int nb, const rst_target* const* src, const rst_target* const* tgt,
                     const rst_icp_opts* opts, const float* poses_in);
int icp_finish_batch(rst_ctx* ctx, float* poses_inout, float* mean_costs, int32_t* status, int32_t* iters);
int icp_align_prepared(rst_ctx* ctx, const rst_target* src,
                       const rst_target* tgt, const rst_icp_opts* opts,
                       float pose_inout[16], float* mean_cost,
                       int32_t* iters_run, rst_comm* comm);
// SolveKabsch (align_icp.cpp:18-71) on device clouds: the means as the
// reference's fp32 sequential sums over the pairs (seqsum.hip); ws holds
// solve_kabsch_ws_bytes(k)
size_t solve_kabsch_ws_bytes(int64_t k);
int solve_kabsch_device(rst_ctx* ctx, const float* d_src, const float* d_dst,
                        const int32_t* d_pairs, const float* d_w, int64_t k, void* ws,
                        float pose_out[16]);
// ComputeCentroid's sums (point_cloud_utils.cpp:94-96) of device xyz:
// out[0..3) = the fp32 sequential sums (host memory); ws holds
// centroid_ws_bytes(n)
size_t centroid_ws_bytes(int64_t n);
int centroid_seq_device(rst_ctx* ctx, const float* d_xyz, int64_t n, void* ws, float out[3]);
int centroid_device(rst_ctx* ctx, const float4* d_pts, int64_t n,
                    double* d_out3);
int seq_sum4_device(rst_ctx* ctx, const float4* d_x, int64_t n, float* d_out);
// the same sums, parallel and bit-exact (seqsum.hip): out[c] for c < nch;
// ws holds seqsum_bytes(n).  stages: bits 1 / 2 / 4 the map pipeline's
// front / maps / walk; with all three, streams of <= RST_SQ_SERIAL_MAX
// elements take the one-wavefront replay (k_sq_serial) instead, unless
// kSqForceMaps; kSqForceSerial takes it at any size; streams of <= 16384
// elements take the one-workgroup-per-chain kernel (k_sq_small), forced by
// kSqForceSmall.
constexpr int kSqForceSerial = 16, kSqForceMaps = 32, kSqForceSmall = 64;
size_t seqsum_bytes(int64_t n);
// a stretch of a longer chain (the sharded loop's relay, comm.hip): per chain
// the fp64 prefix before the stretch (guesses only) and the chain's value at
// its start (device pointers, 4 each); tot_done: seqsum_totals ran on this
// workspace for the same iteration
struct SqStretch {
  const double* p0;
  const float* s0;
  bool tot_done;
};
int seqsum_enqueue(const float4* d_x, int64_t n, int nch, void* ws, float* d_out,
                   hipStream_t st, int* d_stats = nullptr, int stages = 7, int iter = -1,
                   bool fused = false, const SqStretch* stretch = nullptr,
                   unsigned long long* tl = nullptr, int* d_guard = nullptr);
// diagnostics: err bits every walk adds (0 = off), to test the guard path
int seqsum_debug_fault(int bits);
// the sequential sums' DPP wave scan on 64 doubles (in[0..64)), and the block
// scan on in[64..128): out[0..64) inclusive, out[64..128) exclusive, out[128] total
int seqsum_debug_wave_scan(hipStream_t st, const double* h_in, double* h_out);
// a batch of streams summed by one set of launches (the batched ICP loop):
// a device array of records, one per stream (seqsum_pair_fill writes one
// into host memory: the stream, its length, its workspace of
// seqsum_bytes(n), its 4-float output), the chains' count and iteration per
// launch; nmax = the longest stream.  Always the map pipeline.
size_t seqsum_pair_bytes();
void seqsum_pair_fill(void* rec, const float4* d_x, int64_t n, void* ws, float* d_out, unsigned long long* tl,
                      int* d_guard = nullptr);
int seqsum_enqueue_batch(const void* d_pairs, int nbatch, int64_t nmax, int nch, int iter, hipStream_t st,
                         int nch_prev);
// a stretch's fp64 chain totals (d_tot4[4], non-finite elements skipped)
// for the relay's exchange; leaves the quarter totals for seqsum_enqueue
int seqsum_totals(const float4* d_x, int64_t n, int nch, void* ws, double* d_tot4, hipStream_t st,
                  int iter);
int kabsch_device(rst_ctx* ctx, const double cov[9], const float smean[3],
                  const float dmean[3], float pose_out[16]);

// unprojection (unproject.hip)
int unproject_device(rst_ctx* ctx, const uint16_t* d_depth,
                     const rst_intrinsics* K, int keep_invalid,
                     float* d_xyz, int64_t* n_out, int stride = 1,
                     int32_t* d_pixmap = nullptr);

// RemoveNans / DownsampleVoxel (voxel.hip); synchronous (n_out is host)
int remove_nans_device(rst_ctx* ctx, const float* d_xyz, int64_t n, float* d_out,
                       int64_t* n_out);
int downsample_voxel_device(rst_ctx* ctx, const float* d_xyz, int64_t n, float voxel,
                            float* d_out, int64_t* n_out);

// GICP covariances (gicp.hip): d_covs m x 9, original order, col-major 3x3
int compute_covariances_device(rst_ctx* ctx, const rst_target* tgt, int use_gicp,
                               float* d_covs);

// RCCL (comm.hip)
int comm_allreduce_sum_f64(rst_comm* comm, double* d_buf, size_t count,
                           hipStream_t stream);
int comm_size(const rst_comm* comm);
// every rank's shard size (exchanged per layout, checked on the device every
// align): n_total, this rank's offset in the whole source's order, the count
// it runs with, the counts
int comm_shard_layout(rst_comm* comm, int64_t n_local, int64_t n_total_hint, hipStream_t st,
                      int64_t* n_total, int64_t* offset, int64_t* n_eff,
                      const std::vector<int64_t>** counts);
// after k_init_state: this align's gathered counts against the cached
// layout, kGuardLayout into *d_guard on a mismatch (every rank alike)
int comm_layout_check(rst_comm* comm, hipStream_t st, int32_t* d_guard);
// after the loop: every rank's guard word ORed into every rank's (one
// all-gather of an int32 per rank), so a bound check that tripped on one
// rank -- the sequential sums' tables, an index guard -- fails the align on
// all of them alike (no rank goes on to a collective the others skip)
int comm_agree_guard(rst_comm* comm, hipStream_t st, int32_t* d_guard);
// the sequential sums of the ranks' consecutive stretches (d_x: this rank's,
// n_local elements) relayed rank to rank: d_out[0..nch) the whole chains'
// sums on every rank; d_drift: 4 doubles carried between iterations (or null)
int comm_relay_seqsum(rst_comm* comm, const float4* d_x, int64_t n_local, int nch, void* sqws,
                      float* d_out, hipStream_t st, double* d_drift, int* d_stats, int iter,
                      int* d_guard = nullptr);

}  // namespace rst
