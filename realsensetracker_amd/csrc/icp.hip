// icp.hip -- the ICP loop of AlignIcp3d (align_icp.cpp:73-167) on MI355X.
//
// Per iteration three launches on one stream, no host round trip:
//   k_icp_nn<Acc>  one source point per thread: transform, exact NN through
//       the leaf adjacency of last iteration's neighbour (rst_bvh.hpp
//       adj_search; cold lanes start from a Morton-code seed), robust
//       weight, fp64 partial sums -> one slab row per block.  Lanes the
//       adjacency cannot certify are queued (per-block segment, in order);
//   k_icp_fb<Acc>  every block scans the per-block queue counts into LDS,
//       then one wavefront per queued query: the cooperative exact search
//       of rst_wave_nn.hpp, partial sums -> one slab row per block;
//   k_reduce_solve<Acc>  one block: fixed-order reduction of both slabs (bitwise
//       reproducible), then thread 0 solves the 3x3 Kabsch (P2POINT_REF)
//       or 6x6 normal equations (P2PLANE) into the device-resident IcpState.
// Multi-GPU: both slabs are first reduced to one row, all-reduced over
// RCCL, and every rank solves the same pose (DESIGN.md "Multi-GPU").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "rst_device.hpp"
#include "rst_wave_nn.hpp"
#include "rst_internal.hpp"

namespace rst {
namespace {

constexpr int kBS = 256;
constexpr int kNP2Point = 16;  // sum w q u^T (9), sum w u (3), sum q (3), sum d2
constexpr int kNP2Plane = 30;  // A (21), b (6), sum w r^2, count, sum d2
// Far-point certificates.  The fallback search keeps the two nearest: its
// answer p at q0 and a lower bound g (the second distance, less a margin)
// on the distance from q0 to every other point.  In a later iteration the
// same source point at q is certified to have p as its exact nearest
// neighbour when |q - p| + |q - q0| < g (triangle inequality: every other
// point lies at >= g - |q - q0| > |q - p| from q; relative margins 1e-5
// cover the float arithmetic, and the strict gap excludes ties), with no
// search.  nnq[i].w carries kCertBit while the certificate of its point
// holds.  Kernel 1 makes certificates for near points too (adj_search2).
#ifndef RST_FB_MIN_WAVES
#define RST_FB_MIN_WAVES 4  // k_icp_fb occupancy target (r01: 128 VGPRs, 4 waves/SIMD; r02: the kernel's paths need 201, the compiler settles at 2 waves/SIMD; forcing 3 spills: 22.8k vs 23.6k it/s)
#endif
constexpr int kCertBit = 1 << 30;
#ifndef RST_BALL_CHUNK_REF
#define RST_BALL_CHUNK_REF 256  // the REF loop's k_icp_fb ball-tile chunk (points): 25 KB less LDS a block (r12 A/B 34.6k -> 35.1k it/s; the fp64 loop at 256 lost 14%, so it keeps 512)
#endif
constexpr int kBallChunkDefault = 512;
#ifndef RST_FB_MIN_WAVES_REF
#define RST_FB_MIN_WAVES_REF 4  // the REF loop's k_icp_fb (r11: 3 vs 4 waves/SIMD 33.8k vs 33.4k it/s batched; the fp64 loop 49.0k vs 50.0k, so it keeps 4; r20j, with the REF k_icp_nn's below: 4)
#endif
#ifndef RST_COLD_FAST
#define RST_COLD_FAST 1
#endif
#ifndef RST_COLD_ADJ2
#define RST_COLD_ADJ2 0
#endif
#ifndef RST_BALL_TILES
#define RST_BALL_TILES 1  // cold iterations: wave-shared branch-and-bound tiles (k_icp_fb)
#endif
#ifndef RST_BALL_ITERS
#define RST_BALL_ITERS 4  // ... in the first iterations of a pair (r02r: iterations 0-3
                          // 1237/531/426/432 us vs 1668/674/568/492 per-lane; later ones lose)
#endif
#ifndef RST_PIX_TILES
#define RST_PIX_TILES 1  // frame targets: exact searches in the target's pixel grid (k_icp_nn)
#endif
#ifndef RST_ROW_PIX
#define RST_ROW_PIX 1  // k_icp_fb's rows scan the pixel window before the leaf adjacency
#endif
#ifndef RST_PIX_ITERS
#define RST_PIX_ITERS (1 << 30)  // k_icp_nn's pixel windows in a pair's first iterations (r02: 24 -> 11.7 ms per pair alone vs 13.2, but 20.7k vs 23.6k it/s with 4 pairs in flight; default: all)
#endif
#ifndef RST_PIX_CHUNK
#define RST_PIX_CHUNK 384  // pixels staged per wave and round (6 KB of LDS per wave; r02: 512 vs 256 same throughput, one pair 13.4 vs 13.9 ms; r12: 384 with the 5-wave hint below, k_icp_nn at 24.6 KB of LDS and 96 VGPRs a block -- five waves a SIMD --, 33.9k -> 34.7k it/s, fp64 50.2k -> 52.3k)
#endif
constexpr int kPixChunk = RST_PIX_CHUNK;
#ifndef RST_NN_COMPACT
#define RST_NN_COMPACT 0  // RST_SUM_REF: k_icp_nn's pixel-window searches compacted over the workgroup (r04h: nn 35.0 -> 38.6 us steady, fb queues longer -- larger union boxes; 15.1k -> 14.5k it/s)
#endif
#ifndef RST_NN_CLK
#define RST_NN_CLK 0  // diagnostics build: k_icp_nn's wave latencies (tools/nn_clock.py)
#endif
#ifndef RST_NN_CLK_ITER
#define RST_NN_CLK_ITER 64
#endif
#ifndef RST_NN_MIN_WAVES
#define RST_NN_MIN_WAVES 5  // k_icp_nn occupancy hint (waves per SIMD; 6 with 320-pixel chunks spilled: 32.9k)
#endif
#ifndef RST_NN_MIN_WAVES_REF
#define RST_NN_MIN_WAVES_REF 6  // ... of the REF loop's (r20j: with 320-pixel chunks, the batched fallback at 4 waves and the leaf maps at 5 workgroups per CU, 41.0k -> 41.8k it/s; 80 VGPRs, 20 B of scratch)
#endif
#ifndef RST_PIX_CHUNK_REF
#define RST_PIX_CHUNK_REF 320  // pixels staged per wave and round, the REF loop (20.5 KB of LDS a block)
#endif
#ifndef RST_NN_WAVEQ
#define RST_NN_WAVEQ 1  // k_icp_nn (no block sums): queue reservations by LDS atomics, no end barrier
#endif
#ifndef RST_CERT_EAGER
#define RST_CERT_EAGER 0  // k_icp_nn: load cert[] beside nnq[] (not after its flag)
#endif
#ifndef RST_SQ_FUSE_FRONT
#define RST_SQ_FUSE_FRONT 0  // REF loop: the front kernel without the totals launch, the previous iteration's tile prefixes (r04b: front + totals 14.5 -> 13.3 us, but the walk +1 ms per pair: stale guesses in the first iterations)
#endif
#ifndef RST_SQ_FUSE_FROM
#define RST_SQ_FUSE_FROM 0  // ... from this iteration on only (0: never; RST_SQ_FUSE_FROM env overrides), once the pose barely moves
#endif
#ifndef RST_PIX_COLD_ITERS
#define RST_PIX_COLD_ITERS 8  // iterations [1, RST_PIX_COLD_ITERS) take the cold windows below (r04a: 4 vs 3, +1.6 %; r10g: 8 vs 4 27.6k vs 27.2k, 6 27.4k)
#endif
#ifndef RST_SEED_SPARSE
#define RST_SEED_SPARSE 3  // cold seeds: a (2R+1)^2 ring of pixel samples besides the 3x3 (proj_seed; r11c: with the iteration-0 windows below 28.3k vs 27.7k it/s)
#endif
#ifndef RST_SEED_STRIDE
#define RST_SEED_STRIDE 4
#endif
#ifndef RST_PIX_MAX_HALF_REF
#define RST_PIX_MAX_HALF_REF 20.0f  // RST_SUM_REF's k_icp_nn window cap (level pixels; RST_PIX_MAX_HALF elsewhere; r11 ab1-ab6 sweep with 8 staging rounds: 4 28.2k, 8 29.2k, 12 30.0k, 16 30.8k, 20 31.1k, 24 31.1k, 32 30.7k it/s)
#endif
#ifndef RST_PIX_CHUNKS
#define RST_PIX_CHUNKS 11  // staging rounds per wave of the steady-state pixel windows (r11: 2 -> 8 with the 20-pixel cap; 11 at 384-pixel chunks)
#endif
#ifndef RST_PIX_COLD_HALF
#define RST_PIX_COLD_HALF 16.0f  // their half-width cap (level pixels)
#endif
#ifndef RST_PIX_COLD_CHUNKS
#define RST_PIX_COLD_CHUNKS 8  // their staging rounds per wave
#endif
#ifndef RST_PIX_I0_HALF
#define RST_PIX_I0_HALF 24.0f  // > 0: a pair's first iteration takes windows of this cap (level pixels; r11c: iteration 0 nn + fb 1,082 -> 825 us a pair, 16 / 20 px 1,120 / 837; without the sparse seeds no gain)
#endif
#ifndef RST_PIX_I0_CHUNKS
#define RST_PIX_I0_CHUNKS 16  // ... over this many staging rounds per wave
#endif
#ifndef RST_DIAG
#define RST_DIAG 0  // 1: per-iteration certificate counters (rst_debug_queue_trace)
#endif
#ifndef RST_LANE_SMALL_N
#define RST_LANE_SMALL_N 150000  // clouds below this keep the 3n/4 lane-mode threshold (720p pyramid coarse levels; r01k A/B 14.0k -> 14.2k it/s)
#endif
#ifndef RST_XCD_REMAP
#define RST_XCD_REMAP 0  // off: r01i A/B 16.2k -> 16.0k it/s, pyramid level-0 k_icp_nn 140 -> 174 us
#endif
// XCD-aware tile order of k_icp_nn (speed only, never correctness): blocks
// are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md), so block b
// takes tile xcd_tile(b) and each XCD walks one contiguous eighth of the
// Morton-ordered source, whose neighbours are one region of the target: its
// lines are fetched into one XCD's L2 instead of all eight.  Bijective for
// any nb; the slab row and queue segment are the tile's, so the sums and
// the queue order are the same as without the remap.  Measured slower: with
// round-robin placement the blocks in flight at any moment cover one compact
// stretch of the Morton order, whose target lines all eight L2s (and the
// MALL) share; the remap spreads them over eight stretches at once.
__device__ __forceinline__ int xcd_tile(int b, int nb) {
#if RST_XCD_REMAP
  const int x = b & 7, j = b >> 3, per = nb >> 3, rem = nb & 7;
  return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + j;
#else
  (void)nb;
  return b;
#endif
}

// nnq position flags: kCertBit (the certificate in cert[] is valid),
// kFarBit (the last search needed more than the leaf adjacency: the next
// search goes straight to the wave-wide deep search)
constexpr int kFarBit = 1 << 29;
#ifndef RST_PIX_DEFER
#define RST_PIX_DEFER 1  // r19b A/B: 35.13k -> 35.70k it/s, k_icp_nn_b 281 -> 274 us
#endif
#if RST_PIX_DEFER
// kIdBit: the neighbour came from a pixel window of a frame target and nnq
// holds its ORIGINAL index, not its sorted position -- k_icp_nn skips the
// window's dependent inverse-map load (pix_resolve), k_icp_fb converts the
// few it reads (nnq_pos).  RefAcc / P2PointAcc only (P2PLANE reads the
// sorted normals at the position).
constexpr int kIdBit = 1 << 28;
constexpr int kPosMask = kIdBit - 1;
#else
constexpr int kIdBit = 0;
constexpr int kPosMask = kFarBit - 1;
#endif
// an nnq word's sorted position (-1 kept; original indices mapped through
// the frame's inverse map)
__device__ __forceinline__ int nnq_pos(int w, const int32_t* __restrict__ inv, int m) {
  if (w < 0) return w;
  const int p = w & kPosMask;
  if (kIdBit && (w & kIdBit)) return (inv && (uint32_t)p < (uint32_t)m) ? inv[p] : m;
  return p;
}
constexpr int kFbBlocks = 2048;  // largest fallback grid (RST_FB_BLOCKS)
constexpr int kFbBatchRef = 64;
constexpr int kFbRefSingle = 1536;  // a single REF align's fallback grid (fb_grid_ref_single)  // a batch's REF fallback grid per pair (fb_grid_batch_ref)
constexpr int kFbDefault = 384;  // fallback grid (r02 sweep, pixel windows in k_icp_nn: 384 -> 26.2k it/s, 256 26.3k, 512 25.8k, 1024 23.5k; 720p 7.0k vs 6.4k, 720p pyramid 137 vs 130 frames/s)
// From a queue of lane_min entries (IcpParams: the cold first iterations,
// where most lanes' last neighbour is far or missing) kernel 2 finishes the
// queries its adjacency search leaves open one lane per query instead of
// one wavefront per query: the per-lane exact search (rst_bvh.hpp
// search_from) issues 64x fewer instructions per query.  Shorter queues
// hold the far points, whose per-lane searches are long chains: the wave
// search wins there (measured r01).
__device__ __forceinline__ Pose3 load_pose(const IcpState* __restrict__ st) {
  Pose3 P;
#pragma unroll
  for (int k = 0; k < 9; ++k) P.r[k] = st->R[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) P.t[k] = st->t[k];
  return P;
}

// ---- centroid ------------------------------------------------------------------
__global__ __launch_bounds__(kBS) void k_centroid_partial(const float4* __restrict__ pts,
                                                          int64_t n,
                                                          double* __restrict__ slab) {
  __shared__ double lds[(kBS / kWave) * 4];
  double v[4] = {0, 0, 0, 0};
  for (int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBS) {
    const float4 p = pts[i];
    v[0] += p.x;
    v[1] += p.y;
    v[2] += p.z;
    v[3] += 1.0;
  }
  block_sum_to_slab<4, kBS>(v, lds, slab + blockIdx.x * 4);
}

// Reduce slab rows (rows1 of slab1, then rows2 of slab2; NV doubles each)
// into out[NV] in a fixed order (bitwise reproducible): each thread sums a
// strided set of rows, then wave shuffles and one LDS pass.  When fb_e is
// given, slab2 holds rows only for the first ceil(*fb_e / waves-per-block)
// fallback blocks (the others had no queue entries).
constexpr int kRedBS = 1024;
template <int NV>
__device__ __forceinline__ void reduce_slab_rows(const double* __restrict__ slab1, int rows1,
                                                 const double* __restrict__ slab2, int rows2,
                                                 const int32_t* __restrict__ fb_e,
                                                 double* __restrict__ red /*[kRedBS/64][NV]*/,
                                                 double* __restrict__ out) {
  if (fb_e) rows2 = min(rows2, (*fb_e + kBS / kWave - 1) / (kBS / kWave));
  double acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.0;
  for (int b = threadIdx.x; b < rows1 + rows2; b += blockDim.x) {
    const double* row = b < rows1 ? slab1 + (int64_t)b * NV : slab2 + (int64_t)(b - rows1) * NV;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] += row[k];
  }
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = wave_sum(acc[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wid * NV + k] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double t = 0.0;
    for (int w = 0; w < (int)blockDim.x / kWave; ++w) t += red[w * NV + threadIdx.x];
    out[threadIdx.x] = t;
  }
  __syncthreads();
}

template <int NV>
__global__ __launch_bounds__(kRedBS) void k_slab_reduce(const double* __restrict__ slab1, int rows1,
                                                        const double* __restrict__ slab2, int rows2,
                                                        const int32_t* __restrict__ fb_e,
                                                        double* __restrict__ out) {
  __shared__ double red[(kRedBS / kWave) * NV];
  reduce_slab_rows<NV>(slab1, rows1, slab2, rows2, fb_e, red, out);
}

struct InitArgs {
  float pose[16];
  float mu0;
  int32_t need_centroid;  // 0 none (P2PLANE), 1 fp64 slab, 2 sequential float sums
  int32_t chain;  // pyramid: start from the pose the previous solve on this state left
  int64_t n;      // source points (all shards)
};

// State initialisation: pose from the caller (or, chained, the previous
// solve's result: its pose, or its initial pose when it failed -- what
// icp_finish would hand back), mu0, centroid: RST_SUM_REF the reference's
// fp32 sequential sum (k_seq_sum4) * float(1.0 / n) (point_cloud_utils.cpp:
// 92-98), RST_SUM_FP64 the fp64 sum / n rounded to float.
__global__ __launch_bounds__(kBS) void k_init_state(const double* __restrict__ cslab, int rows,
                                                    const float* __restrict__ fsum, InitArgs a,
                                                    IcpState* __restrict__ st) {
  __shared__ double red[(kBS / kWave) * 4];
  __shared__ double tot[4];
#if RST_TIMELINE
  for (int i = threadIdx.x; i < kQTrace * kTlKernels; i += blockDim.x) {
    st->tl[0][0][2 * i] = ~0ull;
    st->tl[0][0][2 * i + 1] = 0ull;
  }
#endif
  if (a.need_centroid == 1) reduce_slab_rows<4>(cslab, rows, cslab, 0, nullptr, red, tot);
  if (threadIdx.x == 0) {
    float P[12];  // R col-major, t
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) P[c * 3 + r] = a.pose[c * 4 + r];
    for (int r = 0; r < 3; ++r) P[9 + r] = a.pose[12 + r];
    if (a.chain) {
      const bool failed = st->fail != 0;
      for (int k = 0; k < 9; ++k) P[k] = failed ? st->in_pose[k] : st->R[k];
      for (int k = 0; k < 3; ++k) P[9 + k] = failed ? st->in_pose[9 + k] : st->t[k];
    }
    for (int k = 0; k < 12; ++k) st->in_pose[k] = P[k];
    for (int k = 0; k < 9; ++k) {
      st->R[k] = P[k];
      st->Rd[k] = P[k];
    }
    for (int r = 0; r < 3; ++r) {
      st->t[r] = P[9 + r];
      st->td[r] = P[9 + r];
    }
    if (a.need_centroid == 2) {
      const float f = (float)(1.0 / (double)a.n);  // `*centroid *= (1.0 / n)`: double -> float
      for (int r = 0; r < 3; ++r) st->smean[r] = fsum[r] * f;
    } else if (a.need_centroid == 1) {
      const double n = tot[3] > 0 ? tot[3] : 1.0;
      for (int r = 0; r < 3; ++r) st->smean[r] = (float)(tot[r] / n);
    } else {
      for (int r = 0; r < 3; ++r) st->smean[r] = 0.f;
    }
    st->mu = a.mu0;
    st->iter = 0;
    for (int k = 0; k < kQTrace; ++k) {
      st->qlen[k] = 0;
      for (int j = 0; j < 4; ++j) st->path[k][j] = st->diag[k][j] = 0;
    }
    st->done = 0;
    st->fail = 0;
    st->last_cost = 0.f;
    st->last_xi = 0;
    st->last_cnt = 0;
    st->last_d2 = 0;
    for (int k = 0; k < 4; ++k) st->seq[k] = 0.f;
    // (guard: cleared by the launch before the centroid's sums, which may
    // already have set a bit; a chained pyramid level keeps the levels before)
  }
}

// ---- per-point accumulation policies ---------------------------------------------
struct Uni {  // uniform per-iteration values of the device state
  Pose3 P;
  float mu;
  float sm0, sm1, sm2;
  int it;  // the iteration
};

__device__ __forceinline__ Uni load_uni(const IcpState* __restrict__ st) {
  Uni u;
  u.P = load_pose(st);
  u.mu = st->mu;
  u.sm0 = st->smean[0];
  u.sm1 = st->smean[1];
  u.sm2 = st->smean[2];
  u.it = st->iter;
  return u;
}

constexpr float kPixHalfLone = 4.0f, kRowHalfLone = 6.0f;  // window caps of a lone (sharded) align
struct AccArgs {
  const float4* __restrict__ nrm;  // P2PLANE: target normals, sorted order
  float4* __restrict__ corr;       // RST_SUM_REF: (q, d2) per original source index
  float pmu;                       // P2PLANE: Geman-McClure scale on r^2
  float max_d2;                    // P2PLANE: correspondence rejection
  int32_t pos0;                    // sorted position of dst[0]
  int32_t full_from;               // RST_SUM_REF: from this iteration on every lane writes
                                   // its record (q, d2): the last one, whose cost chain reads d2
  float pix_half;                  // > 0: k_icp_nn's steady-state window cap (level pixels),
  float row_half;                  // k_icp_fb's rows' cap; 0: the build's (RST_PIX_MAX_HALF*)
};

// P2POINT_REF.  Single pass over the correspondences with the source
// centroid known:  cov = sum w (q - dbar)(s - sbar)^T
//                      = sum w q u^T - dbar (sum w u)^T,
// u = s - sbar in float as at align_icp.cpp:129, dbar = sum q / n (:120-122);
// no neighbour -> q = dst[0], d2 = FLT_MAX (the query's untouched outputs).
struct P2PointAcc {
  static constexpr int NV = kNP2Point;  // sum w q u^T (9), sum w u (3), sum q (3), sum d2
  static constexpr int RS = 16;         // slab row stride (doubles; divides kRedBS)
  static constexpr int kFbMinWaves = RST_FB_MIN_WAVES;  // k_icp_fb occupancy
  static constexpr int kFbMinWavesSingle = kFbMinWaves;
  static constexpr int kNnMinWaves = RST_NN_MIN_WAVES;  // k_icp_nn occupancy
  static constexpr int kPixChunk = RST_PIX_CHUNK;       // k_icp_nn's pixel staging
  static constexpr int kBallChunk = kBallChunkDefault;
  static constexpr bool kPubPrefix = true;  // k_queue_prefix publishes the queues' prefixes
  static constexpr bool kCanFinish = false;
  static constexpr bool kSums = true;  // the search kernels write slab rows
  // q = the neighbour's coordinates (the caller has them), bp its sorted
  // position; no neighbour (bp < 0) -> dst[0], d2 = FLT_MAX
  __device__ static void add(double (&v)[NV], const BvhView& bv, const AccArgs& a, const Uni& u,
                             const float4& s, float px, float py, float pz, float bd, int bp,
                             float4 q, bool same = false) {
    (void)px; (void)py; (void)pz;
    const float l = u.mu / (bd + u.mu);  // :116-117
    const float w = l * l;
    if (bp < 0) q = bv.pts[a.pos0];
    const float u0 = s.x - u.sm0, u1 = s.y - u.sm1, u2 = s.z - u.sm2;
    const double dw = (double)w;
    const double wq0 = dw * (double)q.x, wq1 = dw * (double)q.y, wq2 = dw * (double)q.z;
    v[0] += wq0 * u0; v[1] += wq0 * u1; v[2] += wq0 * u2;
    v[3] += wq1 * u0; v[4] += wq1 * u1; v[5] += wq1 * u2;
    v[6] += wq2 * u0; v[7] += wq2 * u1; v[8] += wq2 * u2;
    v[9] += dw * u0; v[10] += dw * u1; v[11] += dw * u2;
    v[12] += q.x; v[13] += q.y; v[14] += q.z;
    v[15] += bd;
  }
};

// P2PLANE (build's own mode): r = n.(p - q), w = (mu/(r^2+mu))^2,
// J = [p x n ; n]; 21 + 6 + 3 sums.
struct P2PlaneAcc {
  static constexpr int NV = kNP2Plane;  // A (21), b (6), sum w r^2, count, sum d2
  static constexpr int RS = 32;
  static constexpr int kFbMinWaves = 2;  // (unconstrained, the r19 DPP reductions took it to 256 VGPRs and one wave a SIMD: 720p point-to-plane 3.26k -> 2.72k it/s)
  static constexpr int kFbMinWavesSingle = kFbMinWaves;
  static constexpr int kNnMinWaves = RST_NN_MIN_WAVES;
  static constexpr int kPixChunk = RST_PIX_CHUNK;
  static constexpr int kBallChunk = kBallChunkDefault;
  static constexpr bool kPubPrefix = false;  // k_icp_fb scans the queue counts per block (see there)
  static constexpr bool kCanFinish = true;
  static constexpr bool kSums = true;
  __device__ static void add(double (&v)[NV], const BvhView& bv, const AccArgs& a, const Uni& u,
                             const float4& s, float px, float py, float pz, float bd, int bp,
                             float4 q, bool same = false) {
    (void)u; (void)s; (void)bv;
    if (bp < 0 || !(bd <= a.max_d2)) return;
    const float4 nn = a.nrm[bp];
    const float e0 = px - q.x, e1 = py - q.y, e2 = pz - q.z;
    const float r = (nn.x * e0 + nn.y * e1) + nn.z * e2;
    const double dr = (double)r;
    const double l = (double)a.pmu / (dr * dr + (double)a.pmu);
    const double w = l * l;
    const double X = px, Y = py, Z = pz, NX = nn.x, NY = nn.y, NZ = nn.z;
    const double J[6] = {Y * NZ - Z * NY, Z * NX - X * NZ, X * NY - Y * NX, NX, NY, NZ};
    int k = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double wa = w * J[i];
#pragma unroll
      for (int c = 0; c <= i; ++c) v[k++] += wa * J[c];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) v[21 + i] += w * J[i] * dr;
    v[27] += w * dr * dr;
    v[28] += 1.0;
    v[29] += bd;
  }
};

// P2POINT_REF with RST_SUM_REF: the search kernels only record source
// point i's correspondence -- q = dst[nbr_i] (dst[0] when there is none,
// the query's untouched output) and d2 -- at its ORIGINAL index, so that
// k_seq_sum4 can replay the reference's sequential float sums over i
// ascending (align_icp.cpp:105-122) and k_cov_ref its covariance
// (:125-136).  Nothing is summed in the search kernels.
struct RefAcc {
  static constexpr int NV = 9;   // k_cov_ref's rows: the 3x3 covariance
  static constexpr int RS = 16;
  static constexpr int kFbMinWaves = RST_FB_MIN_WAVES_REF;
  static constexpr int kFbMinWavesSingle = 3;  // (the single align's, r11 / r19)
  static constexpr int kNnMinWaves = RST_NN_MIN_WAVES_REF;
  static constexpr int kPixChunk = RST_PIX_CHUNK_REF;
  static constexpr int kBallChunk = RST_BALL_CHUNK_REF;  // k_icp_fb's ball-tile staging (points)
  static constexpr bool kPubPrefix = true;
  static constexpr bool kCanFinish = false;
  static constexpr bool kSums = false;
  __device__ static void add(double (&v)[NV], const BvhView& bv, const AccArgs& a, const Uni& u,
                             const float4& s, float px, float py, float pz, float bd, int bp,
                             float4 q, bool same = false) {
    (void)v; (void)px; (void)py; (void)pz;
    // a lane whose neighbour is the one it had (certified, or found again)
    // leaves its record alone: q is there already, and k_cov_ref recomputes
    // d2 from the pose (every iteration writing every record was 16 B per
    // point of scattered writes, ~26 B per point of write traffic, r05 PMC);
    // the last iteration writes them all, the cost chain reads d2
    if (same && u.it < a.full_from) return;
    if (bp < 0) q = bv.pts[a.pos0];
    a.corr[f2i(s.w)] = make_float4(q.x, q.y, q.z, bd);
  }
};

// ---- RST_SUM_REF: the reference's sequential float32 sums ---------------------------
// One wavefront; lane c < 4 carries chain c (x, y, z, w of a float4 stream)
// through fl(s + x_i) for i ascending from s = +0 -- the order and rounding
// of `dst_mean += dst.GetPoint(j)` / `cost += dist_sqr` (align_icp.cpp:113,
// 120) and of ComputeCentroid's loop (point_cloud_utils.cpp:94-96).  The
// chain is inherently serial (one dependent v_add_f32 per element); the
// wave only keeps it fed: tiles of 64 x kSeqT float4 are loaded coalesced a
// tile ahead and transposed through LDS so lane c reads four of its values
// per ds_read_b128.  out[0..3] = the four sums.
constexpr int kSeqT = 16;                   // float4 per lane per tile (1024 elements)
constexpr int kSeqRow = kSeqT * kWave + 4;  // floats per chain row (+4: rows on distinct banks)
__device__ __forceinline__ void seq_tile_load(const float4* __restrict__ x, int64_t n,
                                              int64_t base, float4 (&v)[kSeqT]) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int t = 0; t < kSeqT; ++t) {
    const int64_t i = base + (int64_t)t * kWave + lane;
    v[t] = i < n ? x[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// transpose one tile through LDS and run lane c's chain over its cnt values
__device__ __forceinline__ void seq_tile_sum(const float4 (&v)[kSeqT], int cnt, float* tile,
                                             float& acc) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int t = 0; t < kSeqT; ++t) {
    tile[0 * kSeqRow + t * kWave + lane] = v[t].x;
    tile[1 * kSeqRow + t * kWave + lane] = v[t].y;
    tile[2 * kSeqRow + t * kWave + lane] = v[t].z;
    tile[3 * kSeqRow + t * kWave + lane] = v[t].w;
  }
  wave_sync();
  if (lane < 4) {
    const float* row = tile + lane * kSeqRow;
    int j = 0;
    for (; j + 4 <= cnt; j += 4) {
      const float4 q = *reinterpret_cast<const float4*>(row + j);
      acc = acc + q.x;
      acc = acc + q.y;
      acc = acc + q.z;
      acc = acc + q.w;
    }
    for (; j < cnt; ++j) acc = acc + row[j];
  }
  wave_sync();
}

__global__ __launch_bounds__(kWave) void k_seq_sum4(const float4* __restrict__ x, int64_t n,
                                                    float* __restrict__ out) {
  __shared__ float4 tile4[4 * kSeqRow / 4];
  float* tile = reinterpret_cast<float*>(tile4);
  constexpr int64_t kT = kSeqT * kWave;
  float acc = 0.0f;
  float4 a[kSeqT], b[kSeqT];
  seq_tile_load(x, n, 0, a);
  for (int64_t base = 0; base < n; base += 2 * kT) {
    seq_tile_load(x, n, base + kT, b);  // in flight during a's chain
    seq_tile_sum(a, (int)min<int64_t>(n - base, kT), tile, acc);
    if (base + kT >= n) break;
    seq_tile_load(x, n, base + 2 * kT, a);
    seq_tile_sum(b, (int)min<int64_t>(n - base - kT, kT), tile, acc);
  }
  if (threadIdx.x < 4) out[threadIdx.x] = acc;
}

// src in original order (the reference iterates i ascending; the prepared
// source is Morton-sorted): out[i] = pts[inv[i]].
__global__ __launch_bounds__(kBS) void k_gather_orig(const float4* __restrict__ pts,
                                                     const int32_t* __restrict__ inv, int64_t n,
                                                     float4* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i < n) out[i] = pts[inv[i]];
}

// The covariance of align_icp.cpp:125-136 with the sequential dst_mean:
// cov += double(float(w_i (q_i - dbar)) * float(s_i - sbar)) per
// coefficient -- the reference's float products, summed in fp64 (the sum
// order only moves the last bits of a double).  dbar = seq / float(n)
// (:122); w_i = (mu / (d2_i + mu))^2 (:116-117).  Grid-stride over the
// original order; one 9-double row (stride RefAcc::RS) per block.
// (r03: 128 blocks measured no faster with pairs in flight and 1.6 us
// slower alone; r06o, batched: 256 blocks 25.6k vs 25.2k ICP it/s -- a
// batch's launch is 256 x B blocks, and the solve reduces 256 rows, not
// 1024; every GPU test bit-identical)
#ifndef RST_COV_BLOCKS
#define RST_COV_BLOCKS 256
#endif
constexpr int kCovBlocks = RST_COV_BLOCKS;
#ifndef RST_COV_UNROLL
#define RST_COV_UNROLL 4
#endif
constexpr int kCovU = RST_COV_UNROLL;
// the covariance grid of a cloud of n points: kCovBlocks, or for small clouds
// (<= 32768 points, the reference callers' 5 cm voxels) ~8 points a thread --
// the solve then reduces a few rows (the fp64 sum order, i.e. the last bits of
// a double, follows n alone: a pair's batched and single aligns agree)
__host__ __device__ __forceinline__ int cov_blocks(int64_t n) {
  return n > 32768 ? kCovBlocks : (int)((n + 8 * kBS - 1) / (8 * kBS)) + (n == 0 ? 1 : 0);
}
// the batched loop launches kCovBlocks blocks per pair and its solve reads
// cov_blocks(n) rows: the small-cloud grid (<= 32768 / (8 kBS) = 16 blocks)
// must fit in it
static_assert(kCovBlocks >= (32768 + 8 * kBS - 1) / (8 * kBS), "RST_COV_BLOCKS below the small-cloud grid");
__device__ __forceinline__ void cov_ref_body(const float4* __restrict__ srco, const float4* __restrict__ corr,
                                             int64_t n, int64_t n_total, const IcpState* __restrict__ st,
                                             double* __restrict__ slab, int nblk) {
  __shared__ double lds[(kBS / kWave) * 9];
#if RST_TIMELINE
  RST_TL(const_cast<IcpState*>(st)->tl[0][0], st->iter, 6);
#endif
  const float nf = (float)n_total;  // dst_mean /= n (the whole source's n)
  const float dm0 = st->seq[0] / nf, dm1 = st->seq[1] / nf, dm2 = st->seq[2] / nf;
  const float sm0 = st->smean[0], sm1 = st->smean[1], sm2 = st->smean[2];
  const float mu = st->mu;
  const Pose3 P = load_pose(st);
  double v[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) v[k] = 0.0;
  // (the thread's points RST_COV_UNROLL at a time, every load issued before
  // the first product -- the same points in the same order, so the same
  // sums; r20f: the kernel's waves spent 70 % of their cycles waiting)
  const int64_t stride = (int64_t)nblk * kBS;
  for (int64_t i0 = blockIdx.x * (int64_t)kBS + threadIdx.x; i0 < n; i0 += kCovU * stride) {
    float4 sv[kCovU], cv[kCovU];
#pragma unroll
    for (int u = 0; u < kCovU; ++u) {
      const int64_t i = i0 + u * stride;
      sv[u] = i < n ? srco[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      cv[u] = i < n ? corr[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kCovU; ++u) {
      if (i0 + u * stride >= n) break;
      const float4 s = sv[u], c = cv[u];
      // d2 of the search (:112), recomputed: the records of lanes that kept
      // their neighbour are not rewritten (RefAcc::add); the same transform and
      // distance arithmetic, so the same bits; no neighbour -> FLT_MAX
      float px, py, pz;
      xform(P, s.x, s.y, s.z, px, py, pz);
      const float d2 = finite3(px, py, pz) ? d2_ref(px, py, pz, c.x, c.y, c.z) : FLT_MAX;
      const float l = mu / (d2 + mu);
      const float w = l * l;
      const float a0 = w * (c.x - dm0), a1 = w * (c.y - dm1), a2 = w * (c.z - dm2);
      const float b0 = s.x - sm0, b1 = s.y - sm1, b2 = s.z - sm2;
      v[0] += (double)(a0 * b0); v[1] += (double)(a0 * b1); v[2] += (double)(a0 * b2);
      v[3] += (double)(a1 * b0); v[4] += (double)(a1 * b1); v[5] += (double)(a1 * b2);
      v[6] += (double)(a2 * b0); v[7] += (double)(a2 * b1); v[8] += (double)(a2 * b2);
    }
  }
  block_sum_to_slab<9, kBS>(v, lds, slab + (int64_t)blockIdx.x * RefAcc::RS);
}

__global__ __launch_bounds__(kBS) void k_cov_ref(const float4* __restrict__ srco,
                                                 const float4* __restrict__ corr, int64_t n,
                                                 int64_t n_total,
                                                 const IcpState* __restrict__ st,
                                                 double* __restrict__ slab) {
  cov_ref_body(srco, corr, n, n_total, st, slab, (int)gridDim.x);
}

// ---- kernel 1: adjacency search, one point per thread ----------------------------------
// Exclusive prefix of the per-block queue counts (one block, kBS threads):
// pref[b] = entries before block b's segment, pref[nb] = E.  pref may be
// LDS (every fallback block scans the counts itself); st, when given,
// receives E (fb_e) and the queue trace.
__device__ void queue_prefix(const int32_t* __restrict__ qcnt, int nb, int32_t* pref,
                             IcpState* __restrict__ st) {
  __shared__ int part[kBS + 1];
  const int per = (nb + kBS - 1) / kBS;
  const int b0 = threadIdx.x * per;
  int sum = 0;
  for (int b = b0; b < b0 + per && b < nb; ++b) sum += __builtin_nontemporal_load(qcnt + b);
  part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x < kWave) {  // one wave scans the kBS partials, 4 per lane
    const int l = threadIdx.x;
    int a[kBS / kWave], t = 0;
#pragma unroll
    for (int k = 0; k < kBS / kWave; ++k) {
      a[k] = part[l * (kBS / kWave) + k];
      t += a[k];
    }
    int inc = t;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int y = __shfl_up(inc, o, kWave);
      if (l >= o) inc += y;
    }
    int acc = inc - t;
#pragma unroll
    for (int k = 0; k < kBS / kWave; ++k) {
      part[l * (kBS / kWave) + k] = acc;
      acc += a[k];
    }
    if (l == kWave - 1) part[kBS] = inc;
  }
  __syncthreads();
  int acc = part[threadIdx.x];
  for (int b = b0; b < b0 + per && b < nb; ++b) {
    pref[b] = acc;
    acc += __builtin_nontemporal_load(qcnt + b);
  }
  if (threadIdx.x == 0) {
    const int E = part[kBS];
    pref[nb] = E;
    if (st) {
      st->fb_e = E;
      if (st->iter < kQTrace) st->qlen[st->iter] = E;
    }
  }
}

// Both fallback queues' prefixes, once per pair and iteration, into gpref
// (near [0, nb], far [nb + 1, 2 nb + 1]) with the queue trace -- a launch of
// its own between k_icp_nn and k_icp_fb, so that k_icp_fb's blocks do not
// each rebuild them (r07: 384 blocks a pair, most without an entry in the
// steady state, each scanning 2 x 1164 counts).  (A last-block ticket in
// k_icp_nn instead needed an agent-scope release per block -- an L2
// write-back each: k_icp_nn_b 94 -> 950 us, r07d.)
__device__ __forceinline__ void queue_prefix_body(const int32_t* __restrict__ qcnt, int nb,
                                                  IcpState* __restrict__ st) {
  if (st->done) return;  // (converged: k_icp_fb returns at once)
  int32_t* gpref = const_cast<int32_t*>(qcnt) + 2 * nb + 64;
  queue_prefix(qcnt, nb, gpref, st);
  __syncthreads();
  queue_prefix(qcnt + nb, nb, gpref + nb + 1, nullptr);
}
__global__ __launch_bounds__(kBS) void k_queue_prefix(const int32_t* __restrict__ qcnt, int nb,
                                                      IcpState* __restrict__ st) {
  queue_prefix_body(qcnt, nb, st);
}

// Projective seeds (frame targets, cold queries): the query projected
// through the target's pixel grid, the valid points of the 3 x 3 level
// pixels around it offered to r -- candidates near the query where Morton
// order jumps (r02: seed distance p90 0.25 m against 1.07 m for the Morton
// seed alone, 0.14 m for the better of both).  Starts only, never answers.
__device__ __forceinline__ void proj_seed(const BvhView& bv, const PixView& pv, float x, float y,
                                          float z, Best2& r) {
  if (!pv.map || !(z > 0.f)) return;
  const float iz = 1.0f / z;
  const float u = (pv.fx * x * iz + pv.cx) / (float)pv.s;
  const float v = (pv.fy * y * iz + pv.cy) / (float)pv.s;
  if (!(u > -2.f && v > -2.f && u < (float)pv.w + 1.f && v < (float)pv.h + 1.f)) return;
  const int uc = (int)floorf(u + 0.5f), vc = (int)floorf(v + 0.5f);
  int cand[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {  // all map loads first: one latency
    const int uu = uc + k % 3 - 1, vv = vc + k / 3 - 1;
    const bool in = uu >= 0 && vv >= 0 && uu < pv.w && vv < pv.h;
    cand[k] = in ? pv.map[(int64_t)vv * pv.w + uu] : -1;
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int c = cand[k];
    if ((uint32_t)c < (uint32_t)bv.m) {
      const float4 w = bv.pts[c];
      r.offer(d2_ref(x, y, z, w.x, w.y, w.z), f2i(w.w), c);
    }
  }
#if RST_SEED_SPARSE
  // Cold lanes only (iteration 0 / new lanes): a sparse ring of samples
  // stride RST_SEED_STRIDE pixels apart out to RST_SEED_SPARSE strides, so
  // that the seed -- the fallback's first ball -- already sits near the
  // surface point a rotation of a few degrees moved the query onto.  Seeds
  // only bound the search; the answer is the exact search's.
  constexpr int R = RST_SEED_SPARSE, S = RST_SEED_STRIDE, D = 2 * R + 1;
  for (int row = 0; row < D; ++row) {
    const int vv = vc + (row - R) * S;
    if (vv < 0 || vv >= pv.h) continue;
    int cs[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int uu = uc + (k - R) * S;
      cs[k] = (uu >= 0 && uu < pv.w) ? pv.map[(int64_t)vv * pv.w + uu] : -1;
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int c = cs[k];
      if ((uint32_t)c < (uint32_t)bv.m) {
        const float4 w = bv.pts[c];
        r.offer(d2_ref(x, y, z, w.x, w.y, w.z), f2i(w.w), c);
      }
    }
  }
#endif
}

// Per source point the loop keeps its neighbour and certificate:
//   nnq[i]  = (p.x, p.y, p.z, pos | kCertBit?): the last exact neighbour's
//             coordinates and sorted position (-1 = cold);
//   cert[i] = (q0.x, q0.y, q0.z, g), valid under kCertBit: when the query
//             was at q0 every target point but p lay at >= g.
// A query now at q keeps p as its exact neighbour while |q - p| + |q - q0|
// < g (triangle inequality, strict: no tie can arise).
//
// Kernel 1 is a pure stream: every lane tests its certificate from three
// coalesced loads (source point, nnq, cert) -- no search, no dependent
// gather -- and accumulates the certified correspondences; every other
// lane goes to the search queue (in point order, one segment per block).
// The searches run compacted in kernel 2, so no wavefront here waits on
// one lane's search.
// (no occupancy hint: the compiler's own register budget, measured best in
// r02 -- a 5-waves/SIMD target spilled)
// (the body of k_icp_nn / k_icp_nn_b: nbk = this pair's grid, the queue
// segments' count)
template <class Acc>
__device__ __forceinline__ void icp_nn_body(const BvhView& bv, const AdjView& av, const PixView& pv,
                                            const AccArgs& aa, const float4* __restrict__ src, int64_t n,
                                            const IcpState* __restrict__ st, float4* __restrict__ nnq,
                                            float4* __restrict__ cert, int32_t* __restrict__ qbuf,
                                            int32_t* __restrict__ qcnt, double* __restrict__ slab,
                                            const int nbk) {
  (void)av;
#if RST_TIMELINE
  RST_TL(const_cast<IcpState*>(st)->tl[0][0], st->iter, 0);
#endif
  __shared__ double lds[(kBS / kWave) * Acc::NV];
  __shared__ int wq[2][kBS / kWave];
#if RST_PIX_TILES
  __shared__ PixScratch<Acc::kPixChunk> pscr[kBS / kWave];
#endif
#if RST_NN_CLK  // diagnostics build: per wave latency and phases (diag[it][0..3])
  const uint64_t ck0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
  uint64_t ck1 = 0, ck2 = 0;
  uint64_t pck[3] = {0, 0, 0};  // pix_tile_search's phases
  uint64_t* const pckp = pck;
#else
  uint64_t* const pckp = nullptr;
#endif
  const int tb = xcd_tile(blockIdx.x, nbk);
  // the far queue: the second half of qbuf / qcnt
  int32_t* __restrict__ qbuff = qbuf + (int64_t)nbk * kBS;
  int32_t* __restrict__ qcntf = qcnt + nbk;
  if (Acc::kCanFinish && st->done) {  // converged: uniform early exit
    if (threadIdx.x == 0) qcnt[tb] = qcntf[tb] = 0;
    return;
  }
  // A loop without block sums (RefAcc) fills the queues without a workgroup
  // barrier at the end: each wavefront reserves its entries in the block's
  // segments by an LDS atomic and the last one to finish publishes the
  // counts, so a wavefront with no search leaves (and frees its registers)
  // instead of waiting for its workgroup's searches (r20h: such waves spent
  // ~5 us of their ~7 at that barrier).  The entries of a segment are then
  // in wavefront arrival order -- nothing the REF fallback's results depend
  // on (a query's answer is its own; no sums fold over the queue).
  constexpr bool kWaveQ = RST_NN_WAVEQ && !Acc::kSums;
  __shared__ int qacc[3];  // near entries, far entries, wavefronts done
  if constexpr (kWaveQ) {
    if (threadIdx.x == 0) qacc[0] = qacc[1] = qacc[2] = 0;
    __syncthreads();  // (at the start: the workgroup's waves arrive together)
  }
  const Uni u = load_uni(st);
  double v[Acc::NV];
#pragma unroll
  for (int k = 0; k < Acc::NV; ++k) v[k] = 0.0;
  const int64_t i = tb * (int64_t)kBS + threadIdx.x;
  const bool act = i < n;
  const float4 s = act ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 tq = act ? nnq[i] : make_float4(0.f, 0.f, 0.f, i2f(-1));
  const int wb = f2i(tq.w);
  const bool has_cert = wb >= 0 && (wb & kCertBit);
#if RST_CERT_EAGER
  // (the certificate loaded beside nnq, not after its flags: one memory
  // round trip before the test instead of two; unused when the flag is off)
  const float4 c = act ? cert[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#else
  const float4 c = (act && has_cert) ? cert[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#endif
  float px, py, pz;
  xform(u.P, s.x, s.y, s.z, px, py, pz);  // align_icp.cpp:107
  const bool fin = finite3(px, py, pz);
  // :112 exact 1-NN by the certificate
  bool certified = false;
  float dq = FLT_MAX;
  if (act && fin && has_cert) {
    dq = d2_ref(px, py, pz, tq.x, tq.y, tq.z);
    const float dx = px - c.x, dy = py - c.y, dz = pz - c.z;
    const float moved = margin_sqrt((dx * dx + dy * dy) + dz * dz) * 1.00001f;
    certified = margin_sqrt(dq) * 1.00001f + moved + 1e-30f < c.w;
  }
  bool need = act && fin && !certified;
  const bool far = wb >= 0 && (wb & kFarBit);
#if RST_NN_CLK
  ck1 = __builtin_amdgcn_s_memtime();
#endif
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  // the search's seed: the last neighbour, or (cold: the pair's first
  // iteration) the better of the projective and the Morton seed
  float d0 = FLT_MAX;
  float4 cq = make_float4(0.f, 0.f, 0.f, 0.f);
  int cpos = -1;
  if (need && wb < 0) {
    Best2 sd;
    sd.init();
    proj_seed(bv, pv, px, py, pz, sd);
    const int ms = morton_seed(bv, px, py, pz);
    const float4 w = bv.pts[ms];
    sd.offer(d2_ref(px, py, pz, w.x, w.y, w.z), f2i(w.w), ms);
    cpos = sd.pos[0];
    cq = bv.pts[cpos];
    d0 = sd.d[0];
  } else if (need) {
    d0 = has_cert ? dq : d2_ref(px, py, pz, tq.x, tq.y, tq.z);
  }
#if RST_PIX_TILES && RST_NN_COMPACT
  if constexpr (std::is_same<Acc, RefAcc>::value) {  // (RefAcc::add reads only s.w)
    if (pv.map && st->iter < RST_PIX_ITERS && n < (int64_t)1 << 30) {  // (i and two flags in 32 bits)
      // The pixel-window searches compacted over the workgroup: the lanes
      // that still need a search (a few per wavefront in the steady state)
      // listed in point order in LDS, the list searched by as many whole
      // wavefronts as it fills -- one, mostly; the others only stream.
      // (r04: a wavefront per 64 points each searching for its own few
      // lanes kept the pass at ~36 us where its stream takes ~8.)
      __shared__ float4 cl_q[kBS];  // query, seed distance
      __shared__ float4 cl_c[kBS];  // cold seed (point, position)
      __shared__ int cl_i[kBS], cl_o[kBS];
      const float sp = (float)pv.s * pz / fminf(fabsf(pv.fx), fabsf(pv.fy));
      const bool reseed = need && wb >= 0 && !(d0 <= 9.f * sp * sp);
      if (__ballot(reseed) != 0 && reseed) d0 = fminf(d0, pix_seed_d2(pv, px, py, pz));
      const uint64_t nm = __ballot(need);
      if (lane == 0) wq[0][wid] = __popcll(nm);
      __syncthreads();
      int slot = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < kBS / kWave; ++w) {
        slot += w < wid ? wq[0][w] : 0;
        tot += wq[0][w];
      }
      const uint64_t lt = (1ull << lane) - 1ull;
      if (need) {
        slot += __popcll(nm & lt);
        cl_q[slot] = make_float4(px, py, pz, d0);
        cl_c[slot] = make_float4(cq.x, cq.y, cq.z, i2f(cpos));
        // (bit 31: far queue; bit 30: cold)
        cl_i[slot] = (int)i | (far ? (int)0x80000000 : 0) | (wb < 0 ? 0x40000000 : 0);
        cl_o[slot] = f2i(s.w);
      }
      // the certified and the non-finite queries' outputs (their own lanes)
      if (certified)
        Acc::add(v, bv, aa, u, s, px, py, pz, dq, f2i(tq.w) & kPosMask, tq, true);
      else if (act && !fin)
        Acc::add(v, bv, aa, u, s, px, py, pz, FLT_MAX, -1, tq);
      __syncthreads();
      const int j = wid * kWave + lane;
      bool fail = false, jfar = false;
      int ji = 0;
      if (wid * kWave < tot) {  // (uniform per wavefront)
        const bool ea = j < tot;
        const float4 q = ea ? cl_q[j] : make_float4(0.f, 0.f, 0.f, FLT_MAX);
        const int code = ea ? cl_i[j] : 0;
        ji = code & 0x3fffffff;
        jfar = code < 0;
        Best2 pr;
        pr.init();
        float4 pq = make_float4(0.f, 0.f, 0.f, 0.f);
        float prc = 0.f;
        const bool cold = st->iter >= 1 && st->iter < RST_PIX_COLD_ITERS;
        const bool pok =
            cold ? pix_tile_search<Acc::kPixChunk, RST_PIX_COLD_CHUNKS>(bv, pv, ea, q.x, q.y, q.z, q.w, pr, pq,
                                                                   pscr[wid], prc, RST_PIX_COLD_HALF)
                 : pix_tile_search<Acc::kPixChunk, RST_PIX_CHUNKS>(bv, pv, ea, q.x, q.y, q.z, q.w, pr, pq, pscr[wid], prc);
        if (pok) {
          const float g = cert_bound(pr, prc);
          const int pos = pr.pos[0];
          nnq[ji] = make_float4(pq.x, pq.y, pq.z, i2f(pos | (g > 0.f ? kCertBit : 0)));
          if (g > 0.f) cert[ji] = make_float4(q.x, q.y, q.z, g);
          const float4 so = make_float4(0.f, 0.f, 0.f, i2f(cl_o[j]));  // (RefAcc: the original index)
          Acc::add(v, bv, aa, u, so, q.x, q.y, q.z, pr.d[0], pos, pq);
        }
        fail = ea && !pok;
        // cold: k_icp_fb starts from nnq's position
        if (fail && (code & 0x40000000)) nnq[ji] = cl_c[j];
#if RST_DIAG
        const uint64_t pm = __ballot(pok);
        if (lane == 0 && st->iter < kQTrace)
          atomicAdd(&const_cast<IcpState*>(st)->diag[st->iter][2], __popcll(pm));
#endif
      }
      // the failures to the queues, in point order
      const uint64_t bm = __ballot(fail && !jfar), fm = __ballot(fail && jfar);
      if (lane == 0) {
        wq[0][wid] = __popcll(bm);
        wq[1][wid] = __popcll(fm);
      }
      __syncthreads();
      int before = 0, total = 0, beforef = 0, totalf = 0;
#pragma unroll
      for (int w = 0; w < kBS / kWave; ++w) {
        before += w < wid ? wq[0][w] : 0;
        total += wq[0][w];
        beforef += w < wid ? wq[1][w] : 0;
        totalf += wq[1][w];
      }
      if (fail && !jfar) qbuf[tb * (int64_t)kBS + before + __popcll(bm & lt)] = ji;
      if (fail && jfar) qbuff[tb * (int64_t)kBS + beforef + __popcll(fm & lt)] = ji;
      if (threadIdx.x == 0) {
        qcnt[tb] = total;
        qcntf[tb] = totalf;
      }
#if RST_DIAG
      const uint64_t cm = __ballot(act && certified);
      if (lane == 0 && st->iter < kQTrace) atomicAdd(&const_cast<IcpState*>(st)->path[st->iter][0], __popcll(cm));
#endif
      return;
    }
  }
#endif
#if RST_PIX_TILES
  // frame target (uniform): the pixel-window search, exact where it
  // applies.  (RST_PIX_ITERS limits it to a pair's first iterations, the
  // few uncertified points of the steady state then go to k_icp_fb's rows:
  // a lower latency per pair, a lower throughput with pairs in flight.)
  if (pv.map && st->iter < RST_PIX_ITERS) {
    Best2 pr;
    pr.init();
    float4 pq = make_float4(0.f, 0.f, 0.f, 0.f);
    float prc = 0.f;
    // a warm seed that moved away: the points around the query's projection
    const float sp = (float)pv.s * pz / fminf(fabsf(pv.fx), fabsf(pv.fy));
    const bool reseed = need && wb >= 0 && !(d0 <= 9.f * sp * sp);
    if (__ballot(reseed) != 0 && reseed) d0 = fminf(d0, pix_seed_d2(pv, px, py, pz));
    // a pair's iterations 1-3: larger windows over more
    // staging rounds (the pose still moves by centimetres, beyond the steady
    // state's cap, which would queue them for k_icp_fb's per-lane searches).
    // The first takes windows up to RST_PIX_I0_HALF pixels: its seeds, the
    // sparse ring around the projection (proj_seed), lie within a few pixels
    // of the neighbour (r03u, with 3 x 3 seeds only, k_icp_fb's ball tiles
    // answered that whole queue faster: 1.06 vs 1.97 ms)
    const bool cold = st->iter >= 1 && st->iter < RST_PIX_COLD_ITERS;
    // (the REF loop's steady-state windows capped smaller: the pass waits on
    // its slowest wavefronts, whose few wide windows the queue's row
    // searches take in parallel instead; r04j: nn 35 -> 25 us, same
    // throughput.  The fp64 loop keeps the wider cap, r02's throughput best)
    constexpr float kPixHalfDef = std::is_same<Acc, RefAcc>::value ? RST_PIX_MAX_HALF_REF : RST_PIX_MAX_HALF;
    const float kPixHalf = aa.pix_half > 0.f ? aa.pix_half : kPixHalfDef;
#if RST_NN_CLK
    ck2 = __builtin_amdgcn_s_memtime();  // (the search's entry, after the reseed)
#endif
    bool pok;
    constexpr bool defer = RST_PIX_DEFER && !std::is_same<Acc, P2PlaneAcc>::value;
    if (RST_PIX_I0_HALF > 0.0f && st->iter == 0)  // (uniform)
      pok = pix_tile_search<Acc::kPixChunk, RST_PIX_I0_CHUNKS, !defer>(bv, pv, need, px, py, pz, d0, pr, pq, pscr[wid],
                                                                  prc, RST_PIX_I0_HALF);
    else if (cold)
      pok = pix_tile_search<Acc::kPixChunk, RST_PIX_COLD_CHUNKS, !defer>(bv, pv, need, px, py, pz, d0, pr, pq,
                                                                        pscr[wid], prc, RST_PIX_COLD_HALF);
    else {
      // (few small windows: the row mode, pix_row_search; else the staged
      // union box)
      bool rows = false;
      if (RST_PIX_ROWMODE && std::is_same<Acc, RefAcc>::value)
        pok = pix_row_search<!defer>(bv, pv, need, px, py, pz, d0, pr, pq, prc, kPixHalf, rows);
      if (!rows)
        pok = pix_tile_search<Acc::kPixChunk, RST_PIX_CHUNKS, !defer>(bv, pv, need, px, py, pz, d0, pr, pq,
                                                                      pscr[wid], prc, kPixHalf, pckp);
    }
    if (pok) {
      const float g = cert_bound(pr, prc);
      // (deferred: the original index, kIdBit -- compared with the last
      // word in the same form; a changed form counts as a change)
      const int pos = defer ? (pr.id[0] | kIdBit) : pr.pos[0];
      nnq[i] = make_float4(pq.x, pq.y, pq.z, i2f(pos | (g > 0.f ? kCertBit : 0)));
      if (g > 0.f) cert[i] = make_float4(px, py, pz, g);
      Acc::add(v, bv, aa, u, s, px, py, pz, pr.d[0], pos, pq, wb >= 0 && pos == (wb & (kPosMask | kIdBit)));
      need = false;
    }
#if RST_DIAG
    const uint64_t pm = __ballot(act && fin && !certified && !need);
    if (lane == 0 && st->iter < kQTrace)
      atomicAdd(&const_cast<IcpState*>(st)->diag[st->iter][2], __popcll(pm));
#endif
  }
#endif
  const uint64_t bm = __ballot(need && !far), fm = __ballot(need && far);
#if RST_DIAG
  {  // diagnostics build: per iteration, lanes certified
    const uint64_t cm = __ballot(act && certified);
    const int it = st->iter;
    if (lane == 0 && it < kQTrace) atomicAdd(&const_cast<IcpState*>(st)->path[it][0], __popcll(cm));
  }
#endif
  const uint64_t lt = (1ull << lane) - 1ull;
  int before = 0, beforef = 0;
  if constexpr (kWaveQ) {
    if (lane == 0) {
      before = atomicAdd(&qacc[0], __popcll(bm));
      beforef = atomicAdd(&qacc[1], __popcll(fm));
    }
    before = __builtin_amdgcn_readfirstlane(before);
    beforef = __builtin_amdgcn_readfirstlane(beforef);
  } else {
    if (lane == 0) {
      wq[0][wid] = __popcll(bm);
      wq[1][wid] = __popcll(fm);
    }
    __syncthreads();
    int total = 0, totalf = 0;
#pragma unroll
    for (int w = 0; w < kBS / kWave; ++w) {
      before += w < wid ? wq[0][w] : 0;
      total += wq[0][w];
      beforef += w < wid ? wq[1][w] : 0;
      totalf += wq[1][w];
    }
    if (threadIdx.x == 0) {
      qcnt[tb] = total;
      qcntf[tb] = totalf;
    }
  }
  if (need && !far) qbuf[tb * (int64_t)kBS + before + __popcll(bm & lt)] = (int)i;
  // cold: k_icp_fb starts from nnq's position
  if (need && wb < 0) nnq[i] = make_float4(cq.x, cq.y, cq.z, i2f(cpos));
  if (need && far) qbuff[tb * (int64_t)kBS + beforef + __popcll(fm & lt)] = (int)i;
  if constexpr (kWaveQ) {
    // the last wavefront publishes the counts (every wavefront's reservations
    // returned before its own `done` increment, so they are all in)
    if (lane == 0 && atomicAdd(&qacc[2], 1) == kBS / kWave - 1) {
      qcnt[tb] = atomicAdd(&qacc[0], 0);
      qcntf[tb] = atomicAdd(&qacc[1], 0);
    }
  }
  if (certified)
    Acc::add(v, bv, aa, u, s, px, py, pz, dq, f2i(tq.w) & kPosMask, tq, true);
  else if (act && !fin)  // no neighbour: the query's untouched outputs
    Acc::add(v, bv, aa, u, s, px, py, pz, FLT_MAX, -1, tq);
  if constexpr (Acc::kSums) block_sum_to_slab<Acc::NV, kBS>(v, lds, slab + (int64_t)tb * Acc::RS);
#if RST_NN_CLK
  // (iteration RST_NN_CLK_ITER only, per wave into the slab -- unused by
  // RefAcc's nn pass: four clocks and the realtime start / end;
  // rst_debug_slab reads it.  Same-address atomics from every wave would
  // serialise and dominate the pass.)
  if (lane == 0 && st->iter == RST_NN_CLK_ITER) {
    const uint64_t ck3 = __builtin_amdgcn_s_memtime(), rt3 = __builtin_amdgcn_s_memrealtime();
    int64_t* o = reinterpret_cast<int64_t*>(slab) + (int64_t)tb * 16 + wid * 4;
    o[0] = (int64_t)rt0;
    o[1] = (int64_t)rt3;
    // shader clocks from the wave's start (0: no such phase): to the
    // certificate test | the search's entry (after the reseed) << 32; the
    // first chunk staged | the scans done << 32
    auto rel = [&](uint64_t t) { return t ? (int64_t)(t - ck0) : 0; };
    o[2] = rel(ck1) | (rel(ck2) << 32);
    o[3] = rel(pck[1]) | (rel(pck[2]) << 32);
  }
#endif
}

template <class Acc>
// (the single align's kernels keep the r19 hints: a pair alone is latency,
// and the REF batch's higher occupancy spills -- r21b, a lone pair 25.8 ms)
__global__ __launch_bounds__(kBS, RST_NN_MIN_WAVES) void k_icp_nn(BvhView bv, AdjView av, PixView pv, AccArgs aa,
                                                const float4* __restrict__ src, int64_t n,
                                                const IcpState* __restrict__ st,
                                                float4* __restrict__ nnq,
                                                float4* __restrict__ cert,
                                                int32_t* __restrict__ qbuf,
                                                int32_t* __restrict__ qcnt,
                                                double* __restrict__ slab) {
  icp_nn_body<Acc>(bv, av, pv, aa, src, n, st, nnq, cert, qbuf, qcnt, slab, (int)gridDim.x);
}

// A batch of independent frame pairs in lockstep (icp_launch_batch): one
// launch per loop kernel for the whole batch, pair = blockIdx.z, its
// arguments from a device array.  (The GPU overlaps only a few kernels from
// independent streams -- its dispatch path, tools/kernel_overlap2.py -- so
// pairs in flight on their own streams leave most of the chip idle between
// small latency-bound kernels; one launch over B pairs gives the chip B
// pairs' work at once.)
struct PairArgs {
  BvhView bv;
  AdjView av;
  PixView pv;
  AccArgs aa;
  const float4* src;  // the prepared (sorted) source
  int64_t n;          // its points (this pair's, this rank's)
  int64_t n_total;
  IcpState* st;
  float4* nnq;
  float4* cert;
  int32_t* qbuf;
  int32_t* qcnt;
  double* slab;   // kernel 1's rows
  double* slab2;  // the fallback grid's / the covariance's rows
  const float4* srco;  // RST_SUM_REF: the source in original order
  float4* corr;        // ... the correspondences
  IcpParams prm;
  int32_t nb1;  // k_icp_nn's grid for this pair
  int32_t lane_min;
};

// The batched kernels read their pointers from a device array, and a
// pointer loaded from memory is a generic (flat) one: every load and store
// of the inlined bodies then became flat_load / flat_store (r19: k_icp_nn_b
// 141 flat and 0 global memory instructions; the single-pair k_icp_nn, its
// pointers kernel arguments, 160 global).  A flat access counts on lgkmcnt
// as well as vmcnt, so each LDS or scalar wait in the pixel windows'
// staging (ds_bpermute shuffles, LDS reads) also waited for every memory
// load in flight.  The pointers are read back as global (address space 1)
// pointers instead -- they only ever hold hipMalloc'd memory -- and the
// compiler's address-space inference carries that into the bodies
// (as_glb, rst_device.hpp).
__device__ __forceinline__ BvhView glb(const BvhView& b) {
  BvhView r = b;
  r.pts = as_glb(b.pts);
  r.nodes = as_glb(b.nodes);
  r.codes = as_glb(b.codes);
  r.lstart = as_glb(b.lstart);
  r.pleaf = as_glb(b.pleaf);
  r.bbox = as_glb(b.bbox);
  return r;
}
__device__ __forceinline__ AdjView glb(const AdjView& a) {
  AdjView r = a;
  r.ent = as_glb(a.ent);
  r.reach = as_glb(a.reach);
  r.ent2 = as_glb(a.ent2);
  r.reach2 = as_glb(a.reach2);
  r.ent3 = as_glb(a.ent3);
  r.reach3 = as_glb(a.reach3);
  return r;
}
__device__ __forceinline__ PixView glb(const PixView& v) {
  PixView r = v;
  r.map = as_glb(v.map);
  r.pts = as_glb(v.pts);
  r.inv = as_glb(v.inv);
  return r;
}
__device__ __forceinline__ AccArgs glb(const AccArgs& a) {
  AccArgs r = a;
  r.nrm = as_glb(a.nrm);
  r.corr = as_glb(a.corr);
  return r;
}
// pair z's arguments with every pointer global
__device__ __forceinline__ PairArgs glb_pair(const PairArgs& A) {
  PairArgs r = A;
  r.bv = glb(A.bv);
  r.av = glb(A.av);
  r.pv = glb(A.pv);
  r.aa = glb(A.aa);
  r.src = as_glb(A.src);
  r.st = as_glb(A.st);
  r.nnq = as_glb(A.nnq);
  r.cert = as_glb(A.cert);
  r.qbuf = as_glb(A.qbuf);
  r.qcnt = as_glb(A.qcnt);
  r.slab = as_glb(A.slab);
  r.slab2 = as_glb(A.slab2);
  r.srco = as_glb(A.srco);
  r.corr = as_glb(A.corr);
  return r;
}

template <class Acc>
__global__ __launch_bounds__(kBS, Acc::kNnMinWaves) void k_icp_nn_b(const PairArgs* __restrict__ pa) {
  const PairArgs& A = pa[blockIdx.z];
  if ((int)blockIdx.x >= A.nb1) return;  // (uniform: the grid fits the batch's largest pair)
  icp_nn_body<Acc>(glb(A.bv), glb(A.av), glb(A.pv), glb(A.aa), as_glb(A.src), A.n, as_glb(A.st), as_glb(A.nnq),
                   as_glb(A.cert), as_glb(A.qbuf), as_glb(A.qcnt), as_glb(A.slab), A.nb1);
}

// Kabsch solve (align_icp.cpp:139-151; SolveKabsch :58-69): fp64 SVD,
// R = float(U V^T), reflection fix, t = dmean - R smean, quaternion trip.
// (A warm start from the previous iteration's polar factor -- the polar
// factor of Qp^T cov, near I -- took as many Newton steps: the scaled
// iteration's step count follows the singular values' spread, r03w.)
// (the rare Jacobi SVD fallback out of line, its 3x3s by value: inlined,
// or called with array pointers, it would keep the solve's arrays in memory
// -- one thread's whole solve then waits on LDS / scratch round trips)
struct M3d {
  double a[9];
};
struct M3f {
  float a[9];
};
__device__ __noinline__ M3f kabsch_svd_r(M3d cov) {
  double U[9], S[3], V[9];
  svd3_jacobi(cov.a, U, S, V);
  M3f R;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      const double a0 = RST_M3(U, r, 0) * RST_M3(V, c, 0);
      const double a1 = RST_M3(U, r, 1) * RST_M3(V, c, 1);
      const double a2 = RST_M3(U, r, 2) * RST_M3(V, c, 2);
      RST_M3(R.a, r, c) = (float)(a0 + (a1 + a2));
    }
  return R;
}

__device__ __forceinline__ void kabsch_solve(const double* cov, const float* smean,
                                             const float* dmean, float* Rq, float* t) {
  // R = U V^T: the polar factor (cheap, nonsingular cov), else Jacobi SVD
  double P[9];
  float R[9];
  if (polar3(cov, P)) {
    for (int k = 0; k < 9; ++k) R[k] = (float)P[k];
  } else {
    M3d cv;
    for (int k = 0; k < 9; ++k) cv.a[k] = cov[k];
    const M3f Rs = kabsch_svd_r(cv);
    for (int k = 0; k < 9; ++k) R[k] = Rs.a[k];
  }
  if (det3f(R) < 0) {  // :143-145 (non-standard fix kept on purpose)
    for (int r = 0; r < 3; ++r) RST_M3(R, r, 2) *= -1.0f;
  }
  for (int r = 0; r < 3; ++r) t[r] = dmean[r] - mv_row(R, r, smean[0], smean[1], smean[2]);
  quat_roundtrip(R, Rq);  // :151
}

__global__ void k_kabsch(const double* __restrict__ in /*cov[9] smean[3] dmean[3]*/,
                         float* __restrict__ out /*pose[16] col-major*/) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float sm[3], dm[3], Rq[9], t[3];
  for (int k = 0; k < 3; ++k) {
    sm[k] = (float)in[9 + k];
    dm[k] = (float)in[12 + k];
  }
  kabsch_solve(in, sm, dm, Rq, t);
  for (int c = 0; c < 3; ++c) {
    for (int r = 0; r < 3; ++r) out[c * 4 + r] = Rq[c * 3 + r];
    out[c * 4 + 3] = 0.f;
  }
  for (int r = 0; r < 3; ++r) out[12 + r] = t[r];
  out[15] = 1.f;
}

// ---- SolveKabsch (align_icp.cpp:18-71): correspondences -> pose ----------------------
// Pass 1: the pairs' points in pair order, src[pairs.first] and
// dst[pairs.second] as float4 streams for the sequential sums of :30-32.
__global__ __launch_bounds__(kBS) void k_pairs_gather(const float* __restrict__ src,
                                                      const float* __restrict__ dst,
                                                      const int32_t* __restrict__ pairs, int64_t k,
                                                      float4* __restrict__ gs,
                                                      float4* __restrict__ gd) {
  const int64_t c = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (c >= k) return;
  const int64_t i = pairs[2 * c], j = pairs[2 * c + 1];
  gs[c] = make_float4(src[3 * i], src[3 * i + 1], src[3 * i + 2], 0.f);
  gd[c] = make_float4(dst[3 * j], dst[3 * j + 1], dst[3 * j + 2], 0.f);
}

// Pass 2: the means (float: src_mean /= indices.size() divides by the float
// Scalar, :33-34), then cov += w * double(float((q - dbar)(s - sbar)^T))
// (:36-54) in fp64.  sums = [src sums | dst sums] (the fp32 sequential sums).
__global__ __launch_bounds__(kBS) void k_pairs_cov(const float* __restrict__ src,
                                                   const float* __restrict__ dst,
                                                   const int32_t* __restrict__ pairs,
                                                   const float* __restrict__ weights, int64_t k,
                                                   const float* __restrict__ sums,
                                                   double* __restrict__ slab) {
  __shared__ double lds[(kBS / kWave) * 9];
  const float fk = (float)k;
  const float sm0 = sums[0] / fk, sm1 = sums[1] / fk, sm2 = sums[2] / fk;
  const float dm0 = sums[4] / fk, dm1 = sums[5] / fk, dm2 = sums[6] / fk;
  double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t c = blockIdx.x * (int64_t)kBS + threadIdx.x; c < k;
       c += (int64_t)gridDim.x * kBS) {
    const int64_t i = pairs[2 * c], j = pairs[2 * c + 1];
    const float u[3] = {src[3 * i] - sm0, src[3 * i + 1] - sm1, src[3 * i + 2] - sm2};
    const float q[3] = {dst[3 * j] - dm0, dst[3 * j + 1] - dm1, dst[3 * j + 2] - dm2};
    const double w = weights ? (double)weights[c] : 1.0;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) v[r * 3 + cc] += w * (double)(q[r] * u[cc]);
  }
  block_sum_to_slab<9, kBS>(v, lds, slab + blockIdx.x * 9);
}

// ComputeCentroid's input: device xyz -> float4 (w = 0) for the sequential sums
__global__ __launch_bounds__(kBS) void k_xyz_f4(const float* __restrict__ xyz, int64_t n,
                                                float4* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i < n) out[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 0.f);
}

// Kabsch on the reduced sums (align_icp.cpp:122, 139-151).
__device__ __forceinline__ void p2point_update(const double* tot, const IcpParams& prm, IcpCore* st) {
  const double n = (double)prm.n;
  float dmean[3];
  for (int r = 0; r < 3; ++r) dmean[r] = (float)(tot[12 + r] / n);
  double cov[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      RST_M3(cov, r, c) = tot[r * 3 + c] - (double)dmean[r] * tot[9 + c];
  float Rq[9], t[3];
  kabsch_solve(cov, st->smean, dmean, Rq, t);
  for (int k = 0; k < 9; ++k) st->R[k] = Rq[k];
  for (int k = 0; k < 3; ++k) st->t[k] = t[k];
  st->last_cost = (float)tot[15];
  const int it = st->iter;
  const int next = it + 1;
  st->iter = next;
  // :96-98 -- mu for iteration `next`
  if (next > 0 && prm.anneal_every > 0 && next % prm.anneal_every == 0) st->mu = st->mu / prm.anneal_div;
}

__device__ bool chol6_solve(const double* Ap /*packed lower 21*/, const double* rhs, double* x) {
  double L[6][6];
  int k = 0;
  double A[6][6];
  for (int a = 0; a < 6; ++a)
    for (int c = 0; c <= a; ++c) {
      A[a][c] = Ap[k];
      A[c][a] = Ap[k];
      ++k;
    }
  for (int i = 0; i < 6; ++i) {
    for (int j = 0; j <= i; ++j) {
      double s = A[i][j];
      for (int q = 0; q < j; ++q) s -= L[i][q] * L[j][q];
      if (i == j) {
        if (!(s > 0.0)) return false;
        L[i][i] = sqrt(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
  }
  double y[6];
  for (int i = 0; i < 6; ++i) {
    double s = rhs[i];
    for (int q = 0; q < i; ++q) s -= L[i][q] * y[q];
    y[i] = s / L[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
    for (int q = i + 1; q < 6; ++q) s -= L[q][i] * x[q];
    x[i] = s / L[i][i];
  }
  return true;
}

__device__ void p2plane_update(const double* tot, const IcpParams& prm, IcpCore* st) {
  if (st->done) return;
  const double cnt = tot[28];
  double xi[6];
  double rhs[6];
  for (int a = 0; a < 6; ++a) rhs[a] = -tot[21 + a];
  if (cnt < 6.0 || !chol6_solve(tot, rhs, xi)) {
    st->done = 1;
    st->fail = 1;
    return;
  }
  // dR = exp([omega]x) (Rodrigues), T <- (dR R, dR t + v)
  const double wx = xi[0], wy = xi[1], wz = xi[2];
  const double th = sqrt(wx * wx + wy * wy + wz * wz);
  double A, B;
  if (th < 1e-12) {
    A = 1.0;
    B = 0.5;
  } else {
    A = sin(th) / th;
    B = (1.0 - cos(th)) / (th * th);
  }
  const double K[9] = {0, wz, -wy, -wz, 0, wx, wy, -wx, 0};  // col-major [w]x
  double dR[9];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) {
      double kk = 0;
      for (int l = 0; l < 3; ++l) kk += RST_M3(K, r, l) * RST_M3(K, l, c);
      RST_M3(dR, r, c) = (r == c ? 1.0 : 0.0) + A * RST_M3(K, r, c) + B * kk;
    }
  double nR[9], nt[3];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) {
      double s = 0;
      for (int l = 0; l < 3; ++l) s += RST_M3(dR, r, l) * RST_M3(st->Rd, l, c);
      RST_M3(nR, r, c) = s;
    }
  for (int r = 0; r < 3; ++r) {
    double s = 0;
    for (int l = 0; l < 3; ++l) s += RST_M3(dR, r, l) * st->td[l];
    nt[r] = s + xi[3 + r];
  }
  for (int k = 0; k < 9; ++k) {
    st->Rd[k] = nR[k];
    st->R[k] = (float)nR[k];
  }
  for (int k = 0; k < 3; ++k) {
    st->td[k] = nt[k];
    st->t[k] = (float)nt[k];
  }
  double nx = 0;
  for (int a = 0; a < 6; ++a) nx += xi[a] * xi[a];
  nx = sqrt(nx);
  st->last_xi = nx;
  st->last_cnt = cnt;
  st->last_d2 = tot[29];
  const int it = st->iter;
  st->iter = it + 1;
  if (nx < (double)prm.p2plane_eps) st->done = 1;
}

// RST_SUM_REF: tot = the covariance (row-major sums of k_cov_ref), the means
// and cost from this iteration's sequential sums (align_icp.cpp:122,
// 139-151; `dst_mean /= n` divides by float(n)).
__device__ __forceinline__ void p2point_ref_update(const double* tot, const IcpParams& prm, IcpCore* st) {
  const float nf = (float)prm.n;
  float dmean[3];
  for (int r = 0; r < 3; ++r) dmean[r] = st->seq[r] / nf;
  double cov[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) RST_M3(cov, r, c) = tot[r * 3 + c];
  float Rq[9], t[3];
  kabsch_solve(cov, st->smean, dmean, Rq, t);
  for (int k = 0; k < 9; ++k) st->R[k] = Rq[k];
  for (int k = 0; k < 3; ++k) st->t[k] = t[k];
  st->last_cost = st->seq[3];
  const int next = st->iter + 1;
  st->iter = next;
  if (next > 0 && prm.anneal_every > 0 && next % prm.anneal_every == 0) st->mu = st->mu / prm.anneal_div;
}

template <class Acc>
__device__ __forceinline__ void acc_update(const double* tot, const IcpParams& prm, IcpCore* st) {
  if constexpr (std::is_same<Acc, RefAcc>::value)
    p2point_ref_update(tot, prm, st);
  else if constexpr (std::is_same<Acc, P2PointAcc>::value)
    p2point_update(tot, prm, st);
  else
    p2plane_update(tot, prm, st);
}

// ---- kernel 3: fixed-order reduction of both slabs + the solve ----------------------
// Rows of Acc::RS doubles (RS divides kRedBS): thread t sums column t % RS
// of rows t / RS, t / RS + kRedBS / RS, ... -- coalesced loads, all in
// flight together -- then per column a fixed-order sum over the kRedBS / RS
// partials.  Bitwise reproducible.  The ICP loop passes rows1 = 0: every
// fallback block's row already holds its share of kernel 1's rows
// (k_icp_fb).  Single GPU: thread 0
// solves (align_icp.cpp:122-151); multi-GPU: the row goes to `totals` for
// the RCCL all-reduce and k_solve_only follows.
template <class Acc>
__device__ __forceinline__ void reduce_solve_body(const double* __restrict__ slab1, int rows1,
                                                  const double* __restrict__ slab2, int rows2max,
                                                  const IcpParams& prm, IcpState* __restrict__ st,
                                                  double* __restrict__ totals) {
  constexpr int RS = Acc::RS, PER = kRedBS / RS, NW = kRedBS / kWave;
  static_assert((RS & (RS - 1)) == 0 && RS <= kWave, "rows: a power of two <= 64 doubles");
  __shared__ double red[NW * RS];
  __shared__ double tot[RS];
#if RST_TIMELINE
  RST_TL(st->tl[0][0], st->iter, 7);
#endif
  if (Acc::kCanFinish && st->done) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int rows2 = rows2max;  // every fallback block writes its row (kernel 1's folded in)
  const int t = threadIdx.x, col = t % RS;
  // unrolled so a thread's loads are all in flight before the first add
  // waits (a rolled loop pays one memory latency per row)
  double acc = 0.0;
#pragma unroll 16
  for (int r = t / RS; r < rows1; r += PER) acc += __builtin_nontemporal_load(slab1 + (int64_t)r * RS + col);
#pragma unroll 16
  for (int r = t / RS; r < rows2; r += PER) acc += __builtin_nontemporal_load(slab2 + (int64_t)r * RS + col);
  // fixed-order tree: lanes l, l ^ RS, l ^ 2RS, ... of a wave hold the same
  // column; then the NW waves' partials, in wave order
#pragma unroll
  for (int o = RS; o < kWave; o <<= 1) acc += __shfl_xor(acc, o, kWave);
  if ((t & (kWave - 1)) < RS) red[(t / kWave) * RS + col] = acc;
  __syncthreads();
  if (t < RS) {
    double x = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) x += red[w * RS + t];
    tot[t] = x;
  }
  __syncthreads();
  if (totals) {
    if (t < Acc::NV) totals[t] = tot[t];
  } else if (t == 0) {
    // (loaded here, not before the reduction: staged through LDS during it,
    // r03w, the solve took as long)
    IcpCore core = *static_cast<const IcpCore*>(st);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const int it = core.iter;
    acc_update<Acc>(tot, prm, &core);
    *static_cast<IcpCore*>(st) = core;
    const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
    if (it < kQTrace) {  // diagnostics (rst_debug_queue_trace): 10 ns ticks
      st->path[it][2] = (int)(t1 - t0);
      st->path[it][3] = (int)(t2 - t1);
      if constexpr (std::is_same<Acc, RefAcc>::value)
        for (int k = 0; k < 4; ++k) st->seqtr[it][k] = core.seq[k];
    }
  }
}

template <class Acc>
__global__ __launch_bounds__(kRedBS) void k_reduce_solve(const double* __restrict__ slab1,
                                                         int rows1,
                                                         const double* __restrict__ slab2,
                                                         int rows2max, IcpParams prm,
                                                         IcpState* __restrict__ st,
                                                         double* __restrict__ totals) {
  reduce_solve_body<Acc>(slab1, rows1, slab2, rows2max, prm, st, totals);
}

// Multi-GPU: the all-reduced row -> the same solve on every rank.
template <class Acc>
__global__ void k_solve_only(const double* __restrict__ totals, IcpParams prm,
                             IcpState* __restrict__ st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  IcpCore core = *static_cast<const IcpCore*>(st);
  if (Acc::kCanFinish && core.done) return;
  double tot[Acc::NV];
  for (int k = 0; k < Acc::NV; ++k) tot[k] = totals[k];
  const int it = core.iter;
  acc_update<Acc>(tot, prm, &core);
  *static_cast<IcpCore*>(st) = core;
  if constexpr (std::is_same<Acc, RefAcc>::value)
    if (it < kQTrace)
      for (int k = 0; k < 4; ++k) st->seqtr[it][k] = core.seq[k];
}

// ---- kernel 2: the searches of the queued queries -----------------------------------
// Kernel 1 leaves two queues (block segments in block order; every block
// here rebuilds both prefixes in LDS from the per-block counts): the near
// queue (certificate failed) and the far queue (certificate failed and the
// last search needed more than the leaf adjacency: frame borders,
// occlusions -- points whose neighbour is far and changes every iteration).
//   * cold (queues >= lane_min: the first iterations of a pair): one entry
//     per lane over both queues -- the wave-shared ball tiles in the first
//     RST_BALL_ITERS iterations, else the two-nearest leaf-adjacency search
//     of the lane's last neighbour (rst_wave_nn.hpp adj_search2), then what
//     that does not cover by the lane's own bottom-up walk;
//   * otherwise the near queue one entry per row of 16 lanes (row_adj2: the
//     leaf adjacency at a few memory latencies), what it does not cover
//     finished at once by the whole wave (deep_search), and the far queue
//     one entry per wavefront, from the last wavefront of the grid down (the
//     ones the near queue leaves idle): the two searches run side by side
//     instead of one after the other.
// Wavefront w takes the contiguous near entries [w C, (w + 1) C), C =
// ceil(E / W) rounded up to whole rounds (spatially coherent runs; a short
// steady-state queue spreads over many waves).  Each entry is added by one
// fixed lane, so the slab is reproducible.  Every block then folds kernel
// 1's slab rows b, b + G, ... into its own row, so the solve kernel reduces
// G rows.  Block 0 publishes the near queue length.

// One query, the whole wavefront (r: uniform seeds in, the two nearest out):
// the leaf adjacency (when try1), level-2 then level-3 adjacency with the
// leaves staged in LDS, else the staged BVH walk.  Returns the certificate
// bound; far = the leaf adjacency did not answer.
__device__ __forceinline__ float deep_search(const BvhView& bv, const AdjView& av, bool try1,
                                             float qx, float qy, float qz, Best2& r,
                                             WnnScratch& ws, bool& far) {
  far = true;
  if (try1) {
    const float rc = nn_wave_adj1(bv, av, r.pos[0], qx, qy, qz, r, ws);
    if (margin_sqrt(r.d[0]) * 1.00001f + 1e-30f < rc) {
      far = false;
      return cert_bound(r, rc);
    }
  }
  const int start = r.pos[0];
  if (!nn_wave_adj(bv, av, kAdj2Shift, start, qx, qy, qz, r, ws) &&
      !nn_wave_adj(bv, av, kAdj3Shift, start, qx, qy, qz, r, ws))
    nn_wave_one(bv, start, qx, qy, qz, r, ws);
  return r.d[1] < FLT_MAX ? margin_sqrt(r.d[1]) * 0.99999f : FLT_MAX;
}

// Source index of queue entry e: near entries [0, E), then far ones.
__device__ __forceinline__ int queue_entry(int e, int E, const int* pref, const int* preff,
                                           int nb1, const int32_t* __restrict__ qbuf,
                                           const int32_t* __restrict__ qbuff) {
  const bool f = e >= E;
  const int* p = f ? preff : pref;
  const int x = f ? e - E : e;
  int lo = 0, hi = nb1 - 1;  // block segment holding entry x
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (p[mid] <= x)
      lo = mid;
    else
      hi = mid - 1;
  }
  return (f ? qbuff : qbuf)[lo * (int64_t)kBS + (x - p[lo])];
}

// The outputs of one answered query: its neighbour (+ certificate, far
// flag) and its term of the sums.
template <class Acc>
__device__ __forceinline__ void fb_record(double (&v)[Acc::NV], const BvhView& bv,
                                          const AccArgs& aa, const Uni& u, float4* __restrict__ nnq,
                                          float4* __restrict__ cert, int i, const float4& s,
                                          float px, float py, float pz, const Best2& r, float g,
                                          bool far) {
  const int pos = r.pos[0];
  const bool cok = pos >= 0 && g > 0.f;
  const float4 q = bv.pts[pos >= 0 ? pos : 0];
  nnq[i] = make_float4(q.x, q.y, q.z,
                       i2f(pos < 0 ? pos : (pos | (cok ? kCertBit : 0) | (far ? kFarBit : 0))));
  if (cok) cert[i] = make_float4(px, py, pz, g);
  Acc::add(v, bv, aa, u, s, px, py, pz, r.d[0], pos, q);
}

// per-wave LDS: the deep search's staging or the ball tiles (never both)
template <int C>
union FbScratchT {
  WnnScratch w;
  BallScratchT<C> b;
};

template <class Acc, bool PUB = Acc::kPubPrefix>
__device__ __forceinline__ void icp_fb_body(const BvhView& bv, const AdjView& av, const PixView& pv,
                                            const AccArgs& aa, const float4* __restrict__ src,
                                            IcpState* __restrict__ st, float4* __restrict__ nnq,
                                            float4* __restrict__ cert, const int32_t* __restrict__ qbuf,
                                            const int32_t* __restrict__ qcnt, int nb1, int lane_min,
                                            const double* __restrict__ slab1, double* __restrict__ slab2,
                                            int64_t n) {
  extern __shared__ int pref[];  // [2 (nb1 + 1)]: near prefix, far prefix
#if RST_TIMELINE
  RST_TL(st->tl[0][0], st->iter, 1);
#endif
  int* preff = pref + nb1 + 1;
  const int32_t* __restrict__ qbuff = qbuf + (int64_t)nb1 * kBS;
  const int32_t* __restrict__ qcntf = qcnt + nb1;
  __shared__ double lds[(kBS / kWave) * Acc::NV];
  __shared__ int rtags[kBS / kWave][kWave / 16][kAdjK];  // row_adj2 candidates
  __shared__ FbScratchT<Acc::kBallChunk> scr[kBS / kWave];
  __shared__ int4 left[kBS / kWave][kWave / 16];  // a round's leftovers (i, seeds)
  if (Acc::kCanFinish && st->done) return;  // converged: nothing reads the slabs
  // The queues' prefixes as k_queue_prefix published them (near [0, nb1],
  // far [nb1 + 1, 2 nb1 + 1]); P2PLANE scans them per block instead (r08:
  // with the published prefixes its k_icp_fb_b took 256 VGPRs, one wave a
  // SIMD, 117.6 -> 195 us; the fp64 P2POINT loop measured 45.4k vs 40.9k
  // it/s for publishing)
  int E, EF;
  if constexpr (!PUB) {
    queue_prefix(qcnt, nb1, pref, blockIdx.x == 0 ? st : nullptr);
    __syncthreads();
    queue_prefix(qcntf, nb1, preff, nullptr);
    __syncthreads();
    E = pref[nb1];
    EF = preff[nb1];
  } else {
    const int32_t* __restrict__ gpref = qcnt + 2 * nb1 + 64;
    E = gpref[nb1];
    EF = gpref[2 * nb1 + 1];
  }
#if RST_DIAG
  if (blockIdx.x == 0 && threadIdx.x == 0 && st->iter < kQTrace) st->diag[st->iter][0] = EF;
#endif
  double v[Acc::NV];
#pragma unroll
  for (int k = 0; k < Acc::NV; ++k) v[k] = 0.0;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const bool many = E + EF >= lane_min;  // uniform
#if RST_BALL_TILES
  // the first iterations of a pair (no neighbour yet, or the pose still
  // moving by centimetres): the wave-shared ball tiles
  const bool ball = many && st->iter < RST_BALL_ITERS;
#endif
  const int W = gridDim.x * (kBS / kWave);
  const int gw = blockIdx.x * (kBS / kWave) + wid;
  // cold: one entry per lane over both queues; else the near queue, one
  // entry per row of 16 lanes
  const int EN = many ? E + EF : E;
  const int per = many ? kWave : kWave / 16;
  const int C = ((EN + W - 1) / W + per - 1) / per * per;
  const int e0 = gw * C, e1 = min(EN, e0 + C);
  const Uni u = load_uni(st);
  // One work loop, so the deep search has a single call site (two inlined
  // copies spill): a pending leftover of the last round, else the next
  // round of entries, else this wave's next far entry.  All uniform.
  const int fg0 = W - 1 - gw;  // this wave's far entries: fg0, fg0 + W, ...
  const int nfar = (!many && fg0 < EF) ? (EF - fg0 + W - 1) / W : 0;
  // a block without an entry (most of the grid in the steady state) loads no
  // prefix; without sums to fold (RST_SUM_REF) it is done
  if constexpr (PUB) {
    if (__syncthreads_or(e0 < e1 || nfar > 0)) {
      const int32_t* __restrict__ gpref = qcnt + 2 * nb1 + 64;
      for (int j = threadIdx.x; j < 2 * (nb1 + 1); j += kBS) pref[j] = gpref[j];
      __syncthreads();
    } else if constexpr (!Acc::kSums) {
      return;
    }
  } else if constexpr (!Acc::kSums) {
    // (the small-cloud REF path scans the counts per block above; a block
    // without an entry then has nothing to fold either)
    if (!__syncthreads_or(e0 < e1 || nfar > 0)) return;
  }
  int r0 = e0, nleft = 0, fdone = 0;
  while (true) {
    bool deep = false, try1 = false;
    int di = 0, dp0 = -1, dp1 = -1;
    if (nleft > 0) {  // a leftover of the last round (the leaf adjacency did not cover it)
      --nleft;
      const int4 en = left[wid][nleft];
      di = en.x;
      dp0 = en.y;
      dp1 = en.z;
      deep = true;
    } else if (r0 < e1) {
      const int e = r0 + (many ? lane : lane >> 4);
      const bool has = e < e1;
      const bool lead = many || (lane & 15) == 0;  // the lane that records the entry
      int i = 0;
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      float px = 0.f, py = 0.f, pz = 0.f;
      bool fin = false;
      Best2 r2;
      r2.init();
      bool exact = false;
      float g = 0.f;
      if (has) {
        i = queue_entry(e, E, pref, preff, nb1, qbuf, qbuff);
        if ((uint32_t)i >= (uint32_t)n) {  // index guard (never expected)
          atomicOr(&st->guard, 1);
          i = 0;
        }
        s = src[i];
        xform(u.P, s.x, s.y, s.z, px, py, pz);
        fin = finite3(px, py, pz);  // (kernel 1 queues finite queries only)
        int warm = nnq_pos(f2i(nnq[i].w), pv.inv, bv.m);
        if (warm >= bv.m) {
          atomicOr(&st->guard, 2);
          warm = -1;
        }
        if (warm < 0) warm = morton_seed(bv, px, py, pz);  // (k_icp_nn seeds cold lanes)
        // seeded with the warm point and its sorted neighbour, so the
        // second bound starts finite
        const float4 w = bv.pts[warm];
        r2.offer(d2_ref(px, py, pz, w.x, w.y, w.z), f2i(w.w), warm);
        if (bv.m > 1) {
          const int nb = warm + 1 < bv.m ? warm + 1 : warm - 1;
          const float4 w2 = bv.pts[nb];
          r2.offer(d2_ref(px, py, pz, w2.x, w2.y, w2.z), f2i(w2.w), nb);
        }
      }
#if RST_BALL_TILES
      if (ball) {
        // cold: the wave's queries share one branch-and-bound walk
        float mq = 0.f;
        const bool act = has && fin;
        int gfail = 0, chunks = 0;
        int4 gdet = make_int4(0, 0, 0, 0);
        const bool done =
            ball_tile_search(bv, act, px, py, pz, r2, mq, scr[wid].b, gfail, gdet, chunks);
        // exact: the lane's own ball built the final box (uncapped), or its
        // first lies inside the box anyway
        const float u0 = margin_sqrt(r2.d[0]) * 1.00001f + 4e-6f;  // ball_box's radius
        if (done && act && (u0 <= RST_BALL_CAP || u0 < mq)) {
          g = fminf(r2.d[1] < FLT_MAX ? margin_sqrt(r2.d[1]) * 0.99999f : FLT_MAX, mq);
          exact = true;
        }
#if RST_DIAG
        if (lane == 0 && st->iter < kQTrace) {
          atomicAdd(&st->diag[st->iter][1], chunks);
        }
#endif
        if (gfail && lane == 0) {
          if (atomicOr(&st->guard, 8 * gfail) == 0) {
            st->path[kQTrace - 1][0] = gdet.x;
            st->path[kQTrace - 1][1] = gdet.y;
            st->path[kQTrace - 1][2] = gdet.z;
            st->path[kQTrace - 1][3] = gdet.w;
          }
        }
      } else
#endif
      if (many) {
        if (has) {
          const float rc = adj_search2(bv, av, r2.pos[0], px, py, pz, r2);
          exact = margin_sqrt(r2.d[0]) * 1.00001f + 1e-30f < rc;
          if (exact) g = cert_bound(r2, rc);
        }
      } else {
        const bool act = has && fin;
        // frame targets: the query's pixel window first (rows of 16 lanes)
        float rcp = 0.f;
        const bool pe = RST_ROW_PIX && pv.map &&
                        row_pix(bv, pv, act, px, py, pz, r2, rcp, aa.row_half > 0.f ? aa.row_half : RST_PIX_MAX_HALF);
        const float rc =
            row_adj2(bv, av, act && !pe, r2.pos[0], px, py, pz, r2, rtags[wid][lane >> 4]);
        if (pe) {
          exact = true;
          g = cert_bound(r2, rcp);
        } else {
          exact = act && margin_sqrt(r2.d[0]) * 1.00001f + 1e-30f < rc;
          if (exact) g = cert_bound(r2, rc);
        }
      }
      if (has && lead && exact) fb_record<Acc>(v, bv, aa, u, nnq, cert, i, s, px, py, pz, r2, g, false);
      const bool unres = lead && has && fin && !exact;
#if RST_DIAG
      {  // diagnostics build: entries answered by the adjacency search
        const uint64_t em = __ballot(lead && has && exact);
        const int it = st->iter;
        if (lane == 0 && it < kQTrace) atomicAdd(&st->path[it][1], __popcll(em));
      }
#endif
      if (many) {
        if (unres) {  // cold start: this lane's own exact walk
          Best1 r = r2.first();
#if RST_COLD_ADJ2
          // the level-2 adjacency (nodes of 8 leaves: a reach several times
          // larger) answers many cold queries before the full walk
          if (!adj2_search(bv, av, r.pos, px, py, pz, r))
#endif
          {
            // bottom-up from the best point so far, every ancestor's
            // sibling box loaded up front (one latency, not one per level)
#if RST_COLD_FAST
            search_from_fast(bv, r.pos, px, py, pz, r);
#else
            search(bv, r.pos, px, py, pz, r);
#endif
          }
          const float4 q = bv.pts[r.pos >= 0 ? r.pos : 0];
          nnq[i] = make_float4(q.x, q.y, q.z, i2f(r.pos));
          Acc::add(v, bv, aa, u, s, px, py, pz, r.d, r.pos, q);
        }
      } else {
        // the row leaders the leaf adjacency did not answer: to the deep
        // search, one at a time (rare once far points have their own queue)
        const uint64_t m = __ballot(unres);
        if (unres)
          left[wid][__popcll(m & ((1ull << lane) - 1ull))] = make_int4(i, r2.pos[0], r2.pos[1], 0);
        nleft = __popcll(m);
        wave_sync();
      }
      r0 += per;
    } else if (fdone < nfar) {  // the far queue: one entry per wavefront
      di = queue_entry(E + fg0 + fdone * W, E, pref, preff, nb1, qbuf, qbuff);
      ++fdone;
      try1 = true;
      deep = true;
    } else {
      break;
    }
    if (deep) {
      if ((uint32_t)di >= (uint32_t)n) {  // index guard (never expected)
        if (lane == 0) atomicOr(&st->guard, 4);
        continue;
      }
      const float4 s = src[di];
      float px, py, pz;
      xform(u.P, s.x, s.y, s.z, px, py, pz);
      if (try1) {  // seeds as the lanes': the last neighbour and its sorted neighbour
        int warm = nnq_pos(f2i(nnq[di].w), pv.inv, bv.m);
        if (warm >= bv.m) {
          if (lane == 0) atomicOr(&st->guard, 2);
          warm = -1;
        }
        if (warm < 0) warm = morton_seed(bv, px, py, pz);
        dp0 = warm;
        dp1 = bv.m > 1 ? (warm + 1 < bv.m ? warm + 1 : warm - 1) : -1;
      }
      Best2 rr;
      rr.init();
      if ((uint32_t)dp0 < (uint32_t)bv.m) {
        const float4 w = bv.pts[dp0];
        rr.offer(d2_ref(px, py, pz, w.x, w.y, w.z), f2i(w.w), dp0);
      }
      if ((uint32_t)dp1 < (uint32_t)bv.m) {
        const float4 w = bv.pts[dp1];
        rr.offer(d2_ref(px, py, pz, w.x, w.y, w.z), f2i(w.w), dp1);
      }
      if (rr.pos[0] < 0) {  // (never expected: a queued query always has a seed)
        if (lane == 0) atomicOr(&st->guard, 2);
        continue;
      }
      bool far = true;
      const float gj = deep_search(bv, av, try1, px, py, pz, rr, scr[wid].w, far);
#if RST_DIAG
      if (lane == 0 && st->iter < kQTrace) atomicAdd(&st->diag[st->iter][3], 1);
#endif
      if (lane == 0) fb_record<Acc>(v, bv, aa, u, nnq, cert, di, s, px, py, pz, rr, gj, far);
    }
  }
  if constexpr (Acc::kSums)
    block_sum_to_slab_fold<Acc::NV, kBS>(v, lds, slab2 + (int64_t)blockIdx.x * Acc::RS, slab1, nb1,
                                         Acc::RS, blockIdx.x, gridDim.x);
}

template <class Acc, bool PUB = Acc::kPubPrefix>
__global__ __launch_bounds__(kBS, Acc::kFbMinWavesSingle) void k_icp_fb(BvhView bv, AdjView av, PixView pv,
                                                AccArgs aa,
                                                const float4* __restrict__ src,
                                                IcpState* __restrict__ st,
                                                float4* __restrict__ nnq,
                                                float4* __restrict__ cert,
                                                const int32_t* __restrict__ qbuf,
                                                const int32_t* __restrict__ qcnt, int nb1,
                                                int lane_min, const double* __restrict__ slab1,
                                                double* __restrict__ slab2, int64_t n) {
  icp_fb_body<Acc, PUB>(bv, av, pv, aa, src, st, nnq, cert, qbuf, qcnt, nb1, lane_min, slab1, slab2, n);
}

// the batch forms (PairArgs, pair = blockIdx.z)
__global__ __launch_bounds__(kBS) void k_queue_prefix_b(const PairArgs* __restrict__ pa) {
  const PairArgs A = glb_pair(pa[blockIdx.z]);
  queue_prefix_body(A.qcnt, A.nb1, A.st);
}

template <class Acc>
__global__ __launch_bounds__(kBS, Acc::kFbMinWaves) void k_icp_fb_b(const PairArgs* __restrict__ pa) {
  const PairArgs A = glb_pair(pa[blockIdx.z]);
  icp_fb_body<Acc>(A.bv, A.av, A.pv, A.aa, A.src, A.st, A.nnq, A.cert, A.qbuf, A.qcnt, A.nb1, A.lane_min,
                   A.slab, A.slab2, A.n);
}

__global__ __launch_bounds__(kBS) void k_cov_ref_b(const PairArgs* __restrict__ pa) {
  const PairArgs A = glb_pair(pa[blockIdx.z]);
  const int nb = cov_blocks(A.n);
  if ((int)blockIdx.x >= nb) return;
  cov_ref_body(A.srco, A.corr, A.n, A.n_total, A.st, A.slab2, nb);
}

template <class Acc>
__global__ __launch_bounds__(kRedBS) void k_reduce_solve_b(const PairArgs* __restrict__ pa, int rows2max) {
  const PairArgs A = glb_pair(pa[blockIdx.z]);
  const int rows = std::is_same<Acc, RefAcc>::value ? cov_blocks(A.n) : rows2max;
  reduce_solve_body<Acc>(A.slab, 0, A.slab2, rows, A.prm, A.st, nullptr);
}

template <class A>
struct AccTag {
  using type = A;
};

inline int blocks_for(int64_t n) { return (int)std::max<int64_t>(1, (n + kBS - 1) / kBS); }

}  // namespace

int kabsch_device(rst_ctx* ctx, const double cov[9], const float smean[3], const float dmean[3],
                  float pose_out[16]) {
  double* buf = nullptr;
  RST_CHECK(ctx_slab(ctx, sizeof(double) * 64, &buf));
  double h[15];
  for (int k = 0; k < 9; ++k) h[k] = cov[k];
  for (int k = 0; k < 3; ++k) {
    h[9 + k] = smean[k];
    h[12 + k] = dmean[k];
  }
  hipStream_t st = ctx->stream;
  RST_HIP(hipMemcpyAsync(buf, h, sizeof(h), hipMemcpyHostToDevice, st));
  k_kabsch<<<1, 64, 0, st>>>(buf, (float*)(buf + 16));
  RST_HIP(hipGetLastError());
  RST_HIP(hipMemcpyAsync(pose_out, buf + 16, sizeof(float) * 16, hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  return RST_OK;
}

// cov (row-major sums from k_pairs_cov) + the float means -> k_kabsch's input layout
__global__ void k_pairs_pack(const float* __restrict__ sums, const double* __restrict__ tot9,
                             int64_t k, double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) RST_M3(out, r, c) = tot9[r * 3 + c];
  const float fk = (float)k;
  for (int a = 0; a < 3; ++a) {
    out[9 + a] = (double)(sums[a] / fk);
    out[12 + a] = (double)(sums[4 + a] / fk);
  }
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t solve_kabsch_ws_bytes(int64_t k) {
  const size_t kk = (size_t)std::max<int64_t>(k, 1);
  return 2 * align256(sizeof(float4) * kk) + 256 + seqsum_bytes(kk);
}

int solve_kabsch_device(rst_ctx* ctx, const float* d_src, const float* d_dst,
                        const int32_t* d_pairs, const float* d_w, int64_t k, void* ws,
                        float pose_out[16]) {
  const int nb = std::min(1024, blocks_for(k));
  double* slab = nullptr;
  RST_CHECK(ctx_slab(ctx, sizeof(double) * (9 * (size_t)nb + 64), &slab));
  double* tot9 = slab + 9 * (size_t)nb;
  double* packed = tot9 + 16;  // 15 in, 16 floats out
  float4* gs = (float4*)ws;
  float4* gd = (float4*)((char*)ws + align256(sizeof(float4) * (size_t)k));
  float* sums = (float*)((char*)gd + align256(sizeof(float4) * (size_t)k));  // [src 4 | dst 4]
  void* sqws = (char*)sums + 256;
  hipStream_t st = ctx->stream;
  k_pairs_gather<<<blocks_for(k), kBS, 0, st>>>(d_src, d_dst, d_pairs, k, gs, gd);
  // src_mean += src.GetPoint(im.first), dst_mean += ... (:30-32), in pair order
  RST_CHECK(seqsum_enqueue(gs, k, 3, sqws, sums, st));
  RST_CHECK(seqsum_enqueue(gd, k, 3, sqws, sums + 4, st));
  k_pairs_cov<<<nb, kBS, 0, st>>>(d_src, d_dst, d_pairs, d_w, k, sums, slab);
  k_slab_reduce<9><<<1, kRedBS, 0, st>>>(slab, nb, slab, 0, nullptr, tot9);
  k_pairs_pack<<<1, 64, 0, st>>>(sums, tot9, k, packed);
  k_kabsch<<<1, 64, 0, st>>>(packed, (float*)(packed + 16));
  RST_HIP(hipGetLastError());
  RST_HIP(hipMemcpyAsync(pose_out, packed + 16, sizeof(float) * 16, hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  return RST_OK;
}

size_t centroid_ws_bytes(int64_t n) {
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  return align256(sizeof(float4) * nn) + 256 + seqsum_bytes(nn);
}

int centroid_seq_device(rst_ctx* ctx, const float* d_xyz, int64_t n, void* ws, float out[3]) {
  float4* x4 = (float4*)ws;
  float* sums = (float*)((char*)ws + align256(sizeof(float4) * (size_t)n));
  void* sqws = (char*)sums + 256;
  hipStream_t st = ctx->stream;
  k_xyz_f4<<<blocks_for(n), kBS, 0, st>>>(d_xyz, n, x4);
  RST_CHECK(seqsum_enqueue(x4, n, 3, sqws, sums, st));
  RST_HIP(hipGetLastError());
  RST_HIP(hipMemcpyAsync(out, sums, sizeof(float) * 3, hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  return RST_OK;
}

// k_seq_sum4 on a device float4 stream (rst_debug_seq_sum4): d_out[4]
int seq_sum4_device(rst_ctx* ctx, const float4* d_x, int64_t n, float* d_out) {
  k_seq_sum4<<<1, kWave, 0, ctx->stream>>>(d_x, n, d_out);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int centroid_device(rst_ctx* ctx, const float4* d_pts, int64_t n, double* d_out) {
  const int nb = std::min(1024, blocks_for(n));
  k_centroid_partial<<<nb, kBS, 0, ctx->stream>>>(d_pts, n, d_out);
  RST_HIP(hipGetLastError());
  return nb;
}

// Enqueue a whole AlignIcp3d on the context's stream (no host round trip
// on a single GPU); icp_finish waits and reads the result.  Returns RST_OK
// when enqueued, RST_FALSE for the reference's early false (nothing
// enqueued), or an error.
// fallback grid (RST_FB_BLOCKS: tuning knob, <= kFbBlocks)
// the first iteration whose sequential sums take the fused front (no
// totals launch; RST_SQ_FUSE_FROM: tuning knob, <= 0 never)
static int sq_fuse_from() {
  static const int g = [] {
    const char* e = getenv("RST_SQ_FUSE_FROM");
    const int v = e ? atoi(e) : (RST_SQ_FUSE_FRONT ? 1 : RST_SQ_FUSE_FROM);
    return v > 0 ? v : INT_MAX;
  }();
  return g;
}

// a batch's RST_SUM_REF fallback grid per pair (RST_FB_BLOCKS_BATCH): RefAcc
// folds no sums there, so the grid moves no bit, and the batch's pairs fill
// the chip together (r11 sweep, 12-pair batches: 384 32.5k, 128 33.1k, 96
// 33.3k, 64 33.5k it/s -- where one pair alone wants 384 or more: the
// reference-shaped host API 29.8 ms a pair at 384, 48 at 128)
static int fb_grid_batch_ref() {
  static const int g = [] {
    const char* e = getenv("RST_FB_BLOCKS_BATCH");
    const int v = e ? atoi(e) : kFbBatchRef;
    return (v >= 1 && v <= kFbBlocks) ? v : kFbBatchRef;
  }();
  return g;
}

// a single REF align's fallback grid (RST_FB_BLOCKS_REF; RefAcc folds no sums,
// so the grid moves no bit): one large pair alone wants every CU (r12 sweep,
// the reference-shaped host API on 640x480 clouds: 384 blocks 29.8 ms a pair,
// 768 26.6, 1024 25.8, 1536 25.4; the sharded 1M pair 2,651 -> 2,870 it/s)
static int fb_grid_ref_single() {
  static const int g = [] {
    const char* e = getenv("RST_FB_BLOCKS_REF");
    const int v = e ? atoi(e) : kFbRefSingle;
    return (v >= 1 && v <= kFbBlocks) ? v : kFbRefSingle;
  }();
  return g;
}

// a single REF align's window caps (icp_launch; run-time env)
static float single_cap(const char* name, float def) {
  const char* e = getenv(name);
  const float v = e ? (float)atof(e) : def;
  return v >= 0.f && v <= 64.f ? v : def;
}

static int fb_grid_size() {
  static const int g = [] {
    const char* e = getenv("RST_FB_BLOCKS");
    const int v = e ? atoi(e) : kFbDefault;
    return (v >= 1 && v <= kFbBlocks) ? v : kFbBlocks;
  }();
  return g;
}

static int64_t small_fb_n() {
  static const int64_t g = [] {
    const char* e = getenv("RST_SMALL_FB_N");
    return e ? (int64_t)atoll(e) : (int64_t)32768;
  }();
  return g;
}

static IcpParams make_params(const rst_icp_opts& opts, int64_t n_total, int64_t n_local) {
  IcpParams prm;
  prm.n = n_total;
  prm.anneal_every = opts.anneal_every;
  prm.anneal_div = opts.anneal_div;
  prm.p2plane_eps = opts.p2plane_eps;
  prm.p2plane_mu = opts.p2plane_mu;
  prm.p2plane_max_d2 = opts.p2plane_max_dist > 0 ? opts.p2plane_max_dist * opts.p2plane_max_dist
                                                 : FLT_MAX;
  prm.max_iter = opts.max_iter;
  prm.sum_mode = opts.sum_mode;
  // queue length from which the fallback runs one lane per query
  // (RST_LANE_MIN_DIV = k: n / k; tuning knob -- r01h sweep: 3n/4 was best;
  // r01j, with queued lanes seeding the fallback: n/3 17.0k, n/4 17.1k, n/2
  // 16.8k, 3n/4 16.6k it/s on the 640x480 stream, the 720p pyramid 14.0k /
  // 13.9k / 14.0k / 14.25k)
  static const int lane_div = [] {
    const char* e = getenv("RST_LANE_MIN_DIV");
    return e ? atoi(e) : 0;
  }();
  // (RST_LANE_MIN_FLOOR: the smallest such queue -- tuning knob)
  static const int lane_floor = [] {
    const char* e = getenv("RST_LANE_MIN_FLOOR");
    return e ? atoi(e) : 16384;
  }();
  prm.lane_min = (int)std::max<int64_t>(
      lane_floor, lane_div > 0 ? n_local / lane_div
                          : (n_local < RST_LANE_SMALL_N ? (3 * n_local) / 4 : n_local / 3));
  return prm;
}

int icp_launch(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
               const rst_icp_opts* opts_in, const float pose_in[16], rst_comm* comm,
               bool chain, int level) {
  if (!ctx || !src || !tgt || !pose_in) return RST_E_ARG;
  if (ctx->bpend.active) return RST_E_STATE;  // one align or batch in flight per context (rst_align.h)
  ctx->pend = {};
  rst_icp_opts opts;
  if (opts_in)
    opts = *opts_in;
  else
    rst_icp_opts_default(&opts);
  const bool p2plane = opts.mode == RST_P2PLANE;
  if (opts.mode != RST_P2POINT_REF && opts.mode != RST_P2PLANE) return RST_E_ARG;
  if (opts.max_iter < 0) return RST_E_ARG;
  if (opts.sum_mode != RST_SUM_REF && opts.sum_mode != RST_SUM_FP64) return RST_E_ARG;
  // the reference's sequential sums (P2POINT_REF only; sharded: the chains
  // are walked over the all-gathered correspondences, comm.hip)
  const bool refsum = !p2plane && opts.sum_mode == RST_SUM_REF;
  if (!tgt->has_bvh) return RST_E_ARG;
  if (tgt->m > kPosMask) return RST_E_ARG;  // positions / indices below the nnq flags
  if (p2plane && !tgt->nrm) return RST_E_STATE;
  int64_t n_local = src->m;
  int64_t n_total = n_local;
  hipStream_t st = ctx->stream;
  // n_total, this shard's offset in the source order and the centroid are
  // global quantities under sharding: the shard layout is exchanged when the
  // caller's n_total asks for it and checked on the device every align
  // (comm.hip); this rank runs with its count of the layout
  int64_t shard_off = 0;  // (the relay needs no offset: every rank keeps its own stretch)
  if (comm) RST_CHECK(comm_shard_layout(comm, src->m, opts.n_total, st, &n_total, &shard_off, &n_local, nullptr));
  // one scratch buffer: [centroid / kernel-1 slab | kernel-2 slab | totals]
  const int nblk = blocks_for(n_local);
  // k_icp_fb scans both queues' per-block counts into dynamic LDS, on top of
  // ~52 KB of static LDS (4 FbScratch + the reductions): 96 KB caps the
  // source at ~3.1M points per align (per shard when sharded)
  if (2 * sizeof(int) * ((size_t)nblk + 1) > (size_t)96 * 1024) return RST_E_ARG;
  const int NV = p2plane ? kNP2Plane : kNP2Point;
  const int RS = p2plane ? P2PlaneAcc::RS : P2PointAcc::RS;
  const int ncb = std::min(1024, blocks_for(n_local));
  // [kernel 1 (+ centroid) | kernel 3 | totals]
  const size_t rows1 = (size_t)std::max(nblk * RS, ncb * 4);
  const size_t slab_doubles = rows1 + (size_t)kFbBlocks * RS + 64;
  double* slab = nullptr;
  RST_CHECK(ctx_slab(ctx, sizeof(double) * slab_doubles, &slab));
  double* slab2 = slab + rows1;
  double* totals = slab2 + (size_t)kFbBlocks * RS;  // 64 doubles

  // reference early return (:77-79): pose untouched
  if (n_total < 3 || tgt->m < 3) return RST_FALSE;
  if (p2plane && n_total < 6) return RST_FALSE;

  // per source point: sorted target position of its last neighbour (warm
  // start of the next iteration's exact search; -1 = cold); the fallback
  // queue (one kBS segment per kernel-1 block) and its per-block counts;
  // RST_SUM_REF: the correspondences and the source in original order (this
  // shard's stretch when sharded: the chains relay rank to rank, comm.hip)
  float4* nnq = nullptr;  // last neighbour (p, pos | kCertBit), -1 = cold
  int32_t *qbuf = nullptr, *qcnt = nullptr;  // near queue, then far queue (k_icp_nn)
  float4* cert = nullptr;  // far-point certificates (read only under kCertBit)
  float4 *corr = nullptr, *srco = nullptr;
  void* sqws = nullptr;  // seqsum.hip tables (RST_SUM_REF)
  {
    const size_t np = (size_t)std::max<int64_t>(n_local, 1);
    const size_t ng = refsum ? np : 0;
    const size_t nq = (size_t)nblk * kBS;
    void* w = nullptr;
    const size_t sqb = refsum ? seqsum_bytes(n_local) : 0;
    RST_CHECK(ctx_workspace(ctx, sizeof(float4) * (2 * np + 2 * ng) + sizeof(int4) * nq +
                                     sizeof(int32_t) * (2 * nq + 4 * nblk + 192) + sqb + 256,
                            &w));
    cert = (float4*)w;
    nnq = cert + np;
    if (refsum) {
      corr = nnq + np;
      srco = corr + ng;
    }
    qbuf = (int32_t*)(cert + 2 * np + 2 * ng);
    qcnt = qbuf + 2 * nq;
    if (refsum)  // the sequential sums' tables (256-byte aligned)
      sqws = (void*)(((uintptr_t)(qcnt + 4 * nblk + 192) + 255) & ~(uintptr_t)255);
    RST_HIP(hipMemsetAsync(nnq, 0xff, sizeof(float4) * np, st));
  }

  if (!chain) RST_HIP(hipMemsetAsync(&ctx->d_state->guard, 0, sizeof(int32_t), st));
  // (walk statistics of this align only: short chains leave theirs zero)
  if (ctx->seq_trace && ctx->d_sqstats && !chain)
    RST_HIP(hipMemsetAsync(ctx->d_sqstats, 0, sizeof(int32_t) * 64 * kQTrace, st));
  InitArgs ia;
  memcpy(ia.pose, pose_in, sizeof(ia.pose));
  ia.mu0 = opts.mu0;
  ia.need_centroid = p2plane ? 0 : (refsum ? 2 : 1);
  ia.chain = chain ? 1 : 0;
  ia.n = n_total;
  int crows = 0;
  float* fsum = (float*)totals;  // RST_SUM_REF: the centroid's sequential sums
  double* drift = totals + 40;   // sharded RST_SUM_REF: the relay's start drift (comm.hip)
  if (refsum) {
    if (n_local > 0) k_gather_orig<<<blocks_for(n_local), kBS, 0, st>>>(src->pts, src->inv, n_local, srco);
    // point_cloud_utils.cpp:94-96 (sharded: the stretches' chains relayed)
    if (comm)
      RST_CHECK(comm_relay_seqsum(comm, srco, n_local, 3, sqws, fsum, st, nullptr, nullptr, -1,
                                  &ctx->d_state->guard));
    else
      RST_CHECK(seqsum_enqueue(srco, n_local, 3, sqws, fsum, st, nullptr, 7, -1, false, nullptr, nullptr,
                               &ctx->d_state->guard));
    k_init_state<<<1, kBS, 0, st>>>(slab, 0, fsum, ia, ctx->d_state);
    if (comm) RST_HIP(hipMemsetAsync(drift, 0, sizeof(double) * 4, st));
  } else if (!p2plane) {
    if (n_local > 0) {
      crows = centroid_device(ctx, src->pts, n_local, slab);
      if (crows < 0) return crows;
    }
    if (comm) {
      k_slab_reduce<4><<<1, kRedBS, 0, st>>>(slab, crows, slab, 0, nullptr, totals);
      RST_CHECK(comm_allreduce_sum_f64(comm, totals, 4, st));
      k_init_state<<<1, kBS, 0, st>>>(totals, 1, nullptr, ia, ctx->d_state);
    } else {
      k_init_state<<<1, kBS, 0, st>>>(slab, crows, nullptr, ia, ctx->d_state);
    }
  } else {
    k_init_state<<<1, kBS, 0, st>>>(slab, 0, nullptr, ia, ctx->d_state);
  }
  if (comm) RST_CHECK(comm_layout_check(comm, st, &ctx->d_state->guard));
  AccArgs aa;
  aa.corr = corr;
  aa.nrm = tgt->nrm;
  aa.pmu = opts.p2plane_mu;
  aa.max_d2 = opts.p2plane_max_dist > 0 ? opts.p2plane_max_dist * opts.p2plane_max_dist : FLT_MAX;
  aa.pos0 = tgt->pos0;
  // (the last iteration's records all written: its cost chain reads d2;
  // every iteration's under the sums' trace)
  aa.full_from = ctx->seq_trace ? 0 : opts.max_iter - 1;
  // the window caps: the build's wide ones pay where many aligns share the
  // chip (batches, aligns in flight); a sharded align is one large pair alone,
  // latency-bound, and takes the narrow ones (r11: the 1M pair 2,517 it/s with
  // 4 / 6 pixels, 2,267 with 20 / 24)
  // A single REF align takes them too (the batches' 20-px
  // cap made a lone 640x480 pair's steady k_icp_nn 70-93 us, its widest
  // lanes' windows; RefAcc folds no sums, so the cap moves no bit -- the
  // fp64 / point-to-plane loops keep the batch's caps, their single and
  // batched aligns must agree bit for bit).  RST_PIX_HALF_SINGLE /
  // RST_ROW_HALF_SINGLE (run-time env) override them; 0 = the batch caps.
  const bool lone = comm || refsum;
  aa.pix_half = lone ? (comm ? kPixHalfLone : single_cap("RST_PIX_HALF_SINGLE", kPixHalfLone)) : 0.f;
  aa.row_half = lone ? (comm ? kRowHalfLone : single_cap("RST_ROW_HALF_SINGLE", kRowHalfLone)) : 0.f;
  const AdjView av = adj_of(tgt);
  const size_t fb_lds = 2 * sizeof(int) * ((size_t)nblk + 1);

  const int fb_grid = fb_grid_size();
  const IcpParams prm = make_params(opts, n_total, n_local);
  // RST_SUM_REF on a small cloud (<= RST_SMALL_FB_N points): the fallback
  // blocks scan the few queue counts themselves, no prefix launch (RefAcc:
  // no sums, results independent of the grid)
  const bool small_fb = refsum && n_local <= small_fb_n();
  // (the single REF align's grid, fb_grid_ref_single: a grid sized to the
  // cloud -- r10c, 2 blocks per kernel-1 block -- spread the cold iterations'
  // queue over too few waves, 231 vs 111 us a cold iteration)
  const int fb_grid_small = fb_grid_ref_single();

  const BvhView bv = view_of(tgt);
  const bool timing = ctx->timing && opts.max_iter > 0;
  if (timing) {  // four events per timed iteration: k1 | k2 | the rest
    const size_t need = 4 * (size_t)opts.max_iter;
    while (ctx->ev.size() < need) {
      hipEvent_t e;
      RST_HIP(hipEventCreate(&e));
      ctx->ev.push_back(e);
    }
  }
  double* red_out = comm ? totals : nullptr;  // multi-GPU: reduce only
  // hipGraph mode: the iteration loop (+ the state readback) is captured and
  // replayed as one graph; the executable per (iterations, mode) is updated
  // in place with this align's arguments (same topology).  Not with RCCL in
  // the loop or per-iteration events.
  const bool graph = ctx->graphs && !comm && !timing && n_local > 0 && opts.max_iter > 0;
  if (graph) RST_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int it = 0; it < opts.max_iter; ++it) {
    const bool tm = timing && it % ctx->timing_stride == 0;  // sampled iterations
    auto mark = [&](int k) -> int {
      if (tm) RST_HIP(hipEventRecord(ctx->ev[4 * it + k], st));
      return RST_OK;
    };
    RST_CHECK(mark(0));
    if (refsum) {
      // align_icp.cpp:105-151 with the reference's rounding: the searches
      // record (q, d2) at the original index, the sequential sums give
      // dst_mean (:113,122) and -- last iteration only: the reference reads
      // only that one (:104,157) -- the cost (:120), k_cov_ref the
      // covariance of the float products (:125-136)
      if (n_local > 0) {
        k_icp_nn<RefAcc><<<nblk, kBS, 0, st>>>(bv, av, tgt->pix, aa, src->pts, n_local, ctx->d_state,
                                               nnq, cert, qbuf, qcnt, slab);
        RST_CHECK(mark(1));
        if (small_fb) {
          // small clouds (the reference callers' 5 cm voxels): no prefix
          // launch -- each fallback block scans the few queue counts itself
          // (<= 2 x 128 for n <= 32768) and, with no entry, returns (RefAcc
          // folds no sums: the grid moves no bit)
          k_icp_fb<RefAcc, false><<<fb_grid_small, kBS, fb_lds, st>>>(bv, av, tgt->pix, aa, src->pts,
                                                                      ctx->d_state, nnq, cert, qbuf, qcnt, nblk,
                                                                      prm.lane_min, slab, slab2, n_local);
        } else {
          k_queue_prefix<<<1, kBS, 0, st>>>(qcnt, nblk, ctx->d_state);
          k_icp_fb<RefAcc><<<fb_grid_ref_single(), kBS, fb_lds, st>>>(bv, av, tgt->pix, aa, src->pts, ctx->d_state, nnq,
                                                         cert, qbuf, qcnt, nblk, prm.lane_min, slab, slab2,
                                                         n_local);
        }
      } else {
        RST_CHECK(mark(1));
      }
      RST_CHECK(mark(2));
      // (from the second iteration on, the same chains as the iteration before:
      // no totals launch, the front kernel takes that iteration's tile
      // prefixes; the last iteration adds the cost chain, which has none)
      const int nch = it + 1 == opts.max_iter || ctx->seq_trace ? 4 : 3;
      const int nch_prev = it == 0 ? 0 : (it == opts.max_iter || ctx->seq_trace ? 4 : 3);
      int* sqstats = ctx->seq_trace && ctx->d_sqstats && it < kQTrace ? ctx->d_sqstats + 64 * it : nullptr;
      if (comm)
        RST_CHECK(comm_relay_seqsum(comm, corr, n_local, nch, sqws, ctx->d_state->seq, st, drift, sqstats, it,
                                    &ctx->d_state->guard));
      else
        RST_CHECK(seqsum_enqueue(corr, n_local, nch, sqws, ctx->d_state->seq, st, sqstats, 7, it,
                                 it > 0 && it >= sq_fuse_from() && nch <= nch_prev, nullptr,
#if RST_TIMELINE
                                 &ctx->d_state->tl[0][0][0],
#else
                                 nullptr,
#endif
                                 &ctx->d_state->guard));
      if (n_local > 0)
        k_cov_ref<<<cov_blocks(n_local), kBS, 0, st>>>(srco, corr, n_local, n_total, ctx->d_state, slab2);
      k_reduce_solve<RefAcc><<<1, kRedBS, 0, st>>>(slab, 0, slab2, n_local > 0 ? cov_blocks(n_local) : 0, prm,
                                                   ctx->d_state, red_out);
      if (comm) {
        RST_CHECK(comm_allreduce_sum_f64(comm, totals, RefAcc::NV, st));
        k_solve_only<RefAcc><<<1, 64, 0, st>>>(totals, prm, ctx->d_state);
      }
    } else if (n_local > 0) {
      // kernel 1 (certificates), kernel 2 (the queued searches)
      auto nn_pass = [&](auto tag) -> int {
        using Acc = typename decltype(tag)::type;
        k_icp_nn<Acc><<<nblk, kBS, 0, st>>>(bv, av, tgt->pix, aa, src->pts, n_local, ctx->d_state, nnq,
                                            cert, qbuf, qcnt, slab);
        RST_CHECK(mark(1));
        if constexpr (Acc::kPubPrefix) k_queue_prefix<<<1, kBS, 0, st>>>(qcnt, nblk, ctx->d_state);
        k_icp_fb<Acc><<<fb_grid, kBS, fb_lds, st>>>(bv, av, tgt->pix, aa, src->pts, ctx->d_state, nnq, cert,
                                                     qbuf, qcnt, nblk, prm.lane_min, slab, slab2,
                                                     n_local);
        return mark(2);
      };
      if (p2plane) {
        RST_CHECK(nn_pass(AccTag<P2PlaneAcc>{}));
        k_reduce_solve<P2PlaneAcc><<<1, kRedBS, 0, st>>>(slab, 0, slab2, fb_grid, prm,
                                                         ctx->d_state, red_out);
      } else {
        RST_CHECK(nn_pass(AccTag<P2PointAcc>{}));
        k_reduce_solve<P2PointAcc><<<1, kRedBS, 0, st>>>(slab, 0, slab2, fb_grid, prm,
                                                         ctx->d_state, red_out);
      }
    } else {
      RST_CHECK(mark(1));
      RST_CHECK(mark(2));
      // an empty shard still joins the all-reduce with zero partial sums
      RST_HIP(hipMemsetAsync(totals, 0, sizeof(double) * NV, st));
    }
    if (comm && !refsum) {
      RST_CHECK(comm_allreduce_sum_f64(comm, totals, NV, st));
      if (p2plane)
        k_solve_only<P2PlaneAcc><<<1, 64, 0, st>>>(totals, prm, ctx->d_state);
      else
        k_solve_only<P2PointAcc><<<1, 64, 0, st>>>(totals, prm, ctx->d_state);
    }
    RST_CHECK(mark(3));
  }
  RST_HIP(hipGetLastError());
  // sharded: a bound check that tripped on one rank fails the align on every
  // rank (the relay hands the other ranks NaN sums, which alone
  // would read as the reference's false there)
  if (comm) RST_CHECK(comm_agree_guard(comm, st, &ctx->d_state->guard));
  RST_HIP(hipMemcpyAsync(ctx->h_state, ctx->d_state, sizeof(IcpState), hipMemcpyDeviceToHost, st));
  if (graph) {
    hipGraph_t g = nullptr;
    RST_HIP(hipStreamEndCapture(st, &g));
    // one executable per (pyramid level, iterations, kernel sequence): the
    // levels of one pyramid are queued back to back, so a level must never
    // update an executable whose launch for another level is still pending
    hipGraphExec_t& ex = ctx->gexec[std::make_tuple(level, opts.max_iter, (int)p2plane, (int)refsum)];
    if (ex) {
      hipGraphNode_t err_node = nullptr;
      hipGraphExecUpdateResult ur;
      if (hipGraphExecUpdate(ex, g, &err_node, &ur) != hipSuccess ||
          ur != hipGraphExecUpdateSuccess) {
        (void)hipGetLastError();
        hipGraphExecDestroy(ex);
        ex = nullptr;
      }
    }
    if (!ex && hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) {
      ex = nullptr;
      hipGraphDestroy(g);
      return RST_E_HIP;
    }
    hipGraphDestroy(g);
    RST_HIP(hipGraphLaunch(ex, st));
  }
  ctx->pend.active = true;
  ctx->pend.p2plane = p2plane;
  ctx->pend.timing = timing;
  ctx->pend.max_iter = opts.max_iter;
  ctx->pend.n_total = n_total;
  return RST_OK;
}

// a sequential-sum table's bound check tripped (seqsum.hip err bits): the
// sums -- NaN by then -- would read as the reference's false; an internal
// error instead
static int seqsum_guard_error(int32_t guard) {
  static thread_local char msg[160];
  snprintf(msg, sizeof(msg), "sequential-sum bound check tripped (err bits %d): sums not computed",
           (int)((uint32_t)guard >> kGuardSeqsumShift));
  set_last_error(hipErrorIllegalAddress, msg, __FILE__, __LINE__);
  return RST_E_HIP;
}

int icp_finish(rst_ctx* ctx, float pose_inout[16], float* mean_cost, int32_t* iters_run) {
  if (!ctx || !pose_inout) return RST_E_ARG;
  if (!ctx->pend.active) return RST_E_STATE;
  const auto pd = ctx->pend;
  ctx->pend.active = false;
  if (pd.early_false) return RST_FALSE;  // pose untouched (align_icp.cpp:77-79)
  RST_HIP(hipStreamSynchronize(ctx->stream));
  if (pd.timing) {
    float tot[3] = {0.f, 0.f, 0.f};
    int cnt = 0;
    for (int it = 0; it < pd.max_iter; it += ctx->timing_stride) {
      for (int k = 0; k < 3; ++k) {
        float ms = 0.f;
        RST_HIP(hipEventElapsedTime(&ms, ctx->ev[4 * it + k], ctx->ev[4 * it + k + 1]));
        tot[k] += ms;
      }
      ++cnt;
    }
    ctx->last_kernel_ms = cnt ? tot[0] / cnt : 0.f;
    for (int k = 0; k < 3; ++k) ctx->last_iter_ms[k] = cnt ? tot[k] / cnt : 0.f;
    ctx->last_kernel_launches = cnt;
  }
  const IcpState& h = *ctx->h_state;
  ctx->last_iters = h.iter;
  if (h.guard & kGuardLayout) {  // (every rank of the communicator alike)
    set_last_error(hipSuccess, "sharded align: a shard size changed while n_total did not (pass the new "
                   "n_total, or 0, on every rank)", __FILE__, __LINE__);
    return RST_E_ARG;
  }
  if (h.guard & kGuardSeqsum) return seqsum_guard_error(h.guard);
  if (h.guard) {  // an index guard tripped: corrupted queue / neighbour state
    static thread_local char msg[160];
    const int32_t* d = h.path[kQTrace - 1];  // the first trip's details (kernel-specific)
    snprintf(msg, sizeof(msg), "ICP index guard bits %d (detail %d %d %d %d)", h.guard, d[0], d[1],
             d[2], d[3]);
    set_last_error(hipErrorIllegalAddress, msg, __FILE__, __LINE__);
    return RST_E_HIP;
  }
  if (pd.p2plane && h.fail) {
    if (iters_run) *iters_run = h.iter;
    if (pd.pyramid) {  // the pose level 0 started from (the coarser levels' result)
      for (int c = 0; c < 3; ++c) {
        for (int r = 0; r < 3; ++r) pose_inout[c * 4 + r] = h.in_pose[c * 3 + r];
        pose_inout[c * 4 + 3] = 0.f;
      }
      for (int r = 0; r < 3; ++r) pose_inout[12 + r] = h.in_pose[9 + r];
      pose_inout[15] = 1.f;
    }
    return RST_FALSE;
  }
  if (pd.max_iter > 0 || pd.p2plane || pd.pyramid) {  // (a pyramid's coarse levels moved it)
    for (int c = 0; c < 3; ++c) {
      for (int r = 0; r < 3; ++r) pose_inout[c * 4 + r] = h.R[c * 3 + r];
      pose_inout[c * 4 + 3] = 0.f;
    }
    for (int r = 0; r < 3; ++r) pose_inout[12 + r] = h.t[r];
    pose_inout[15] = 1.f;
  }
  if (iters_run) *iters_run = h.iter;
  float mc;
  if (pd.p2plane) {
    mc = h.last_cnt > 0 ? (float)sqrt(h.last_d2 / h.last_cnt) : 0.f;
  } else {
    // :157 mean_cost = sqrt(cost / n) with cost the last iteration's sum d2
    mc = sqrtf(h.last_cost / (float)pd.n_total);
  }
  if (mean_cost) *mean_cost = mc;
  if (pd.p2plane) return RST_OK;
  return (mc < 10000.0f) ? RST_OK : RST_FALSE;  // :160 (NaN -> false)
}

// ---- a batch of frame pairs in lockstep -----------------------------------------------
// The same loop as icp_launch for nb independent pairs at once: per pair its
// own state, workspace and slab; per iteration ONE launch of each loop
// kernel for the whole batch (pair = blockIdx.z, its arguments from a
// device array of PairArgs; the sequential sums from one of SqPair
// records).  Each pair's arithmetic is exactly its icp_launch's (the same
// kernels' bodies, the same grids), so each result is bit-identical to
// aligning it alone.  No RCCL, no hipGraph (plain stream launches).
int icp_launch_batch(rst_ctx* ctx, int nb, const rst_target* const* src, const rst_target* const* tgt,
                     const rst_icp_opts* opts_in, const float* poses_in) {
  if (!ctx || nb < 1 || !src || !tgt || !poses_in) return RST_E_ARG;
  if (ctx->bpend.active || ctx->pend.active) return RST_E_STATE;
  rst_icp_opts opts;
  if (opts_in)
    opts = *opts_in;
  else
    rst_icp_opts_default(&opts);
  const bool p2plane = opts.mode == RST_P2PLANE;
  if (opts.mode != RST_P2POINT_REF && opts.mode != RST_P2PLANE) return RST_E_ARG;
  if (opts.max_iter < 0) return RST_E_ARG;
  if (opts.sum_mode != RST_SUM_REF && opts.sum_mode != RST_SUM_FP64) return RST_E_ARG;
  const bool refsum = !p2plane && opts.sum_mode == RST_SUM_REF;
  hipStream_t st = ctx->stream;
  // the pairs that run (the reference's early false, align_icp.cpp:77-79: left out)
  std::vector<int32_t> slot(nb, -1);
  std::vector<int> run;
  for (int p = 0; p < nb; ++p) {
    if (!src[p] || !tgt[p]) return RST_E_ARG;
    if (!tgt[p]->has_bvh || tgt[p]->m > kPosMask) return RST_E_ARG;
    if (p2plane && !tgt[p]->nrm) return RST_E_STATE;
    const int64_t n = src[p]->m;
    if (n < 3 || tgt[p]->m < 3 || (p2plane && n < 6)) continue;
    slot[p] = (int32_t)run.size();
    run.push_back(p);
  }
  const int B = (int)run.size();
  ctx->bpend = {};
  ctx->bpend.nb = nb;
  ctx->bpend.slot = slot;
  ctx->bpend.n_total.assign(nb, 0);
  ctx->bpend.max_iter = opts.max_iter;
  ctx->bpend.p2plane = p2plane;
  for (int p = 0; p < nb; ++p) ctx->bpend.n_total[p] = src[p]->m;
  if (B == 0) {
    ctx->bpend.active = true;
    return RST_OK;
  }
  // per pair: states
  if (ctx->bcap < B) {
    RST_HIP(hipStreamSynchronize(st));
    if (ctx->d_bstate) hipFree(ctx->d_bstate);
    if (ctx->h_bstate) hipHostFree(ctx->h_bstate);
    ctx->d_bstate = nullptr;
    ctx->h_bstate = nullptr;
    ctx->bcap = 0;
    if (hipMalloc(&ctx->d_bstate, sizeof(IcpState) * B) != hipSuccess ||
        hipHostMalloc(&ctx->h_bstate, sizeof(IcpState) * B, hipHostMallocDefault) != hipSuccess)
      return RST_E_NOMEM;
    ctx->bcap = B;
  }
  RST_HIP(hipMemsetAsync(ctx->d_bstate, 0, sizeof(IcpState) * B, st));  // (every guard word cleared)
  // per pair: slab and workspace sizes (as icp_launch), carved from one of each
  const int NVmode = p2plane ? kNP2Plane : kNP2Point;
  (void)NVmode;
  const int RS = p2plane ? P2PlaneAcc::RS : P2PointAcc::RS;
  const int fb_grid = fb_grid_size();
  std::vector<size_t> slab_off(B), ws_off(B);
  std::vector<int> nblk(B);
  size_t slab_tot = 0, ws_tot = 0;
  int nblk_max = 0;
  int64_t nmax = 1;
  auto a256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
  for (int b = 0; b < B; ++b) {
    const int64_t n = src[run[b]]->m;
    nblk[b] = blocks_for(n);
    nblk_max = std::max(nblk_max, nblk[b]);
    nmax = std::max(nmax, n);
    const int ncb = std::min(1024, blocks_for(n));
    const size_t rows1 = (size_t)std::max(nblk[b] * RS, ncb * 4);
    slab_off[b] = slab_tot;
    slab_tot += a256(sizeof(double) * (rows1 + (size_t)kFbBlocks * RS + 64));
    const size_t np = (size_t)n, ng = refsum ? np : 0, nq = (size_t)nblk[b] * kBS;
    ws_off[b] = ws_tot;
    ws_tot += a256(sizeof(float4) * (2 * np + 2 * ng) + sizeof(int4) * nq + sizeof(int32_t) * (2 * nq + 4 * nblk[b] + 192)) +
              (refsum ? a256(seqsum_bytes(n)) : 0) + 256;
  }
  const size_t fb_lds = 2 * sizeof(int) * ((size_t)nblk_max + 1);
  if (fb_lds > (size_t)96 * 1024) return RST_E_ARG;
  const size_t pa_off = ws_tot, sq_off = a256(pa_off + sizeof(PairArgs) * B);
  const size_t ws_all = a256(sq_off + seqsum_pair_bytes() * B);
  double* slab_all = nullptr;
  void* ws_all_p = nullptr;
  RST_CHECK(ctx_slab(ctx, slab_tot, &slab_all));
  RST_CHECK(ctx_workspace(ctx, ws_all, &ws_all_p));
  char* W = (char*)ws_all_p;
  std::vector<PairArgs> pa(B);
  std::vector<char> sqrec(seqsum_pair_bytes() * B);
  const IcpParams prm0 = make_params(opts, nmax, nmax);
  for (int b = 0; b < B; ++b) {
    const rst_target* S = src[run[b]];
    const rst_target* T = tgt[run[b]];
    const int64_t n = S->m;
    IcpState* dst = ctx->d_bstate + b;
    double* slab = (double*)((char*)slab_all + slab_off[b]);
    const int ncb = std::min(1024, blocks_for(n));
    const size_t rows1 = (size_t)std::max(nblk[b] * RS, ncb * 4);
    double* slab2 = slab + rows1;
    double* totals = slab2 + (size_t)kFbBlocks * RS;
    char* w = W + ws_off[b];
    const size_t np = (size_t)n, ng = refsum ? np : 0, nq = (size_t)nblk[b] * kBS;
    float4* cert = (float4*)w;
    float4* nnq = cert + np;
    float4* corr = refsum ? nnq + np : nullptr;
    float4* srco = refsum ? corr + ng : nullptr;
    int32_t* qbuf = (int32_t*)(cert + 2 * np + 2 * ng);
    int32_t* qcnt = qbuf + 2 * nq;
    void* sqws = refsum ? (void*)(((uintptr_t)(qcnt + 4 * nblk[b] + 192) + 255) & ~(uintptr_t)255) : nullptr;
    RST_HIP(hipMemsetAsync(nnq, 0xff, sizeof(float4) * np, st));
    // init (per pair, once): the source centroid, the state
    InitArgs ia;
    memcpy(ia.pose, poses_in + 16 * run[b], sizeof(ia.pose));
    ia.mu0 = opts.mu0;
    ia.need_centroid = p2plane ? 0 : (refsum ? 2 : 1);
    ia.chain = 0;
    ia.n = n;
    float* fsum = (float*)totals;
    if (refsum) {
      k_gather_orig<<<blocks_for(n), kBS, 0, st>>>(S->pts, S->inv, n, srco);
      RST_CHECK(seqsum_enqueue(srco, n, 3, sqws, fsum, st, nullptr, 7, -1, false, nullptr, nullptr,
                               &dst->guard));  // point_cloud_utils.cpp:94-96
      k_init_state<<<1, kBS, 0, st>>>(slab, 0, fsum, ia, dst);
    } else if (!p2plane) {
      const int crows = centroid_device(ctx, S->pts, n, slab);
      if (crows < 0) return crows;
      k_init_state<<<1, kBS, 0, st>>>(slab, crows, nullptr, ia, dst);
    } else {
      k_init_state<<<1, kBS, 0, st>>>(slab, 0, nullptr, ia, dst);
    }
    PairArgs& A = pa[b];
    A.bv = view_of(T);
    A.av = adj_of(T);
    A.pv = T->pix;
    A.aa.nrm = T->nrm;
    A.aa.corr = corr;
    A.aa.pmu = opts.p2plane_mu;
    A.aa.max_d2 = opts.p2plane_max_dist > 0 ? opts.p2plane_max_dist * opts.p2plane_max_dist : FLT_MAX;
    A.aa.pos0 = T->pos0;
    A.aa.full_from = opts.max_iter - 1;
    A.src = S->pts;
    A.n = n;
    A.n_total = n;
    A.st = dst;
    A.nnq = nnq;
    A.cert = cert;
    A.qbuf = qbuf;
    A.qcnt = qcnt;
    A.slab = slab;
    A.slab2 = slab2;
    A.srco = srco;
    A.corr = corr;
    A.prm = make_params(opts, n, n);
    A.nb1 = nblk[b];
    A.lane_min = A.prm.lane_min;
    if (refsum)
      seqsum_pair_fill(sqrec.data() + seqsum_pair_bytes() * b, corr, n, sqws, dst->seq,
#if RST_TIMELINE
                       &dst->tl[0][0][0],
#else
                       nullptr,
#endif
                       &dst->guard);
  }
  (void)prm0;
  const PairArgs* d_pa = (const PairArgs*)(W + pa_off);
  const void* d_sq = W + sq_off;
  RST_CHECK(stage_h2d(ctx, (void*)d_pa, pa.data(), sizeof(PairArgs) * B));
  if (refsum) RST_CHECK(stage_h2d(ctx, (void*)d_sq, sqrec.data(), sqrec.size()));
  const bool timing = ctx->timing && opts.max_iter > 0;
  if (timing) {
    const size_t need = 4 * (size_t)opts.max_iter;
    while (ctx->ev.size() < need) {
      hipEvent_t e;
      RST_HIP(hipEventCreate(&e));
      ctx->ev.push_back(e);
    }
  }
  const dim3 gnn(nblk_max, 1, B), gfb(fb_grid, 1, B), gone(1, 1, B), gfb_ref(fb_grid_batch_ref(), 1, B);
  for (int it = 0; it < opts.max_iter; ++it) {
    const bool tm = timing && it % ctx->timing_stride == 0;
    auto mark = [&](int k) -> int {
      if (tm) RST_HIP(hipEventRecord(ctx->ev[4 * it + k], st));
      return RST_OK;
    };
    RST_CHECK(mark(0));
    if (refsum) {
      k_icp_nn_b<RefAcc><<<gnn, kBS, 0, st>>>(d_pa);
      RST_CHECK(mark(1));
      k_queue_prefix_b<<<gone, kBS, 0, st>>>(d_pa);
      k_icp_fb_b<RefAcc><<<gfb_ref, kBS, fb_lds, st>>>(d_pa);
      RST_CHECK(mark(2));
      RST_CHECK(seqsum_enqueue_batch(d_sq, B, nmax, it + 1 == opts.max_iter ? 4 : 3, it, st, it > 0 ? 3 : 0));
      k_cov_ref_b<<<dim3(kCovBlocks, 1, B), kBS, 0, st>>>(d_pa);
      k_reduce_solve_b<RefAcc><<<gone, kRedBS, 0, st>>>(d_pa, kCovBlocks);
    } else if (p2plane) {
      k_icp_nn_b<P2PlaneAcc><<<gnn, kBS, 0, st>>>(d_pa);
      RST_CHECK(mark(1));
      k_icp_fb_b<P2PlaneAcc><<<gfb, kBS, fb_lds, st>>>(d_pa);
      RST_CHECK(mark(2));
      k_reduce_solve_b<P2PlaneAcc><<<gone, kRedBS, 0, st>>>(d_pa, fb_grid);
    } else {
      k_icp_nn_b<P2PointAcc><<<gnn, kBS, 0, st>>>(d_pa);
      RST_CHECK(mark(1));
      k_queue_prefix_b<<<gone, kBS, 0, st>>>(d_pa);
      k_icp_fb_b<P2PointAcc><<<gfb, kBS, fb_lds, st>>>(d_pa);
      RST_CHECK(mark(2));
      k_reduce_solve_b<P2PointAcc><<<gone, kRedBS, 0, st>>>(d_pa, fb_grid);
    }
    RST_CHECK(mark(3));
  }
  RST_HIP(hipGetLastError());
  RST_HIP(hipMemcpyAsync(ctx->h_bstate, ctx->d_bstate, sizeof(IcpState) * B, hipMemcpyDeviceToHost, st));
  ctx->bpend.active = true;
  ctx->bpend.timing = timing;
  return RST_OK;
}

// one pair's result from its final state (icp_finish's rules)
static int state_result(const IcpState& h, bool p2plane, int max_iter, int64_t n_total, float pose_inout[16],
                        float* mean_cost, int32_t* iters_run) {
  if (h.guard & kGuardSeqsum) return seqsum_guard_error(h.guard);
  if (h.guard) {
    static thread_local char msg[160];
    const int32_t* d = h.path[kQTrace - 1];
    snprintf(msg, sizeof(msg), "ICP index guard bits %d (detail %d %d %d %d)", h.guard, d[0], d[1], d[2], d[3]);
    set_last_error(hipErrorIllegalAddress, msg, __FILE__, __LINE__);
    return RST_E_HIP;
  }
  if (iters_run) *iters_run = h.iter;
  if (p2plane && h.fail) return RST_FALSE;
  if (max_iter > 0 || p2plane) {
    for (int c = 0; c < 3; ++c) {
      for (int r = 0; r < 3; ++r) pose_inout[c * 4 + r] = h.R[c * 3 + r];
      pose_inout[c * 4 + 3] = 0.f;
    }
    for (int r = 0; r < 3; ++r) pose_inout[12 + r] = h.t[r];
    pose_inout[15] = 1.f;
  }
  const float mc = p2plane ? (h.last_cnt > 0 ? (float)sqrt(h.last_d2 / h.last_cnt) : 0.f)
                           : sqrtf(h.last_cost / (float)n_total);  // :157
  if (mean_cost) *mean_cost = mc;
  if (p2plane) return RST_OK;
  return (mc < 10000.0f) ? RST_OK : RST_FALSE;  // :160 (NaN -> false)
}

int icp_finish_batch(rst_ctx* ctx, float* poses_inout, float* mean_costs, int32_t* status, int32_t* iters) {
  if (!ctx || !poses_inout || !status) return RST_E_ARG;
  if (!ctx->bpend.active) return RST_E_STATE;
  const auto pd = ctx->bpend;
  ctx->bpend.active = false;
  RST_HIP(hipStreamSynchronize(ctx->stream));
  if (pd.timing) {
    float tot[3] = {0.f, 0.f, 0.f};
    int cnt = 0;
    for (int it = 0; it < pd.max_iter; it += ctx->timing_stride) {
      for (int k = 0; k < 3; ++k) {
        float ms = 0.f;
        RST_HIP(hipEventElapsedTime(&ms, ctx->ev[4 * it + k], ctx->ev[4 * it + k + 1]));
        tot[k] += ms;
      }
      ++cnt;
    }
    ctx->last_kernel_ms = cnt ? tot[0] / cnt : 0.f;
    for (int k = 0; k < 3; ++k) ctx->last_iter_ms[k] = cnt ? tot[k] / cnt : 0.f;
    ctx->last_kernel_launches = cnt;
  }
  int worst = RST_OK;
  for (int p = 0; p < pd.nb; ++p) {
    if (mean_costs) mean_costs[p] = 0.f;
    if (iters) iters[p] = 0;
    if (pd.slot[p] < 0) {  // pose untouched (align_icp.cpp:77-79)
      status[p] = RST_FALSE;
      continue;
    }
    status[p] = state_result(ctx->h_bstate[pd.slot[p]], pd.p2plane, pd.max_iter, pd.n_total[p],
                             poses_inout + 16 * p, mean_costs ? mean_costs + p : nullptr, iters ? iters + p : nullptr);
    if (status[p] < 0) worst = status[p];
  }
  return worst;
}

// ---- diagnostics: the sharded loop's two halves (rst_debug.h) ------------------------
// The state a sharded iteration starts from: pose, mu, source centroid and
// iteration count set directly (k_init_state, then these).
__global__ void k_debug_state(IcpState* __restrict__ st, const float* __restrict__ smean, float mu,
                              int iter) {
  if (threadIdx.x != 0) return;
  for (int r = 0; r < 3; ++r) st->smean[r] = smean[r];
  st->mu = mu;
  st->iter = iter;
}

int icp_debug_partials(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
                       const rst_icp_opts* opts_in, const float pose[16], float mu,
                       const float smean[3], int32_t iter, double* out, int32_t* nv) {
  if (!ctx || !src || !tgt || !pose || !smean || !out || !nv) return RST_E_ARG;
  rst_icp_opts opts;
  if (opts_in)
    opts = *opts_in;
  else
    rst_icp_opts_default(&opts);
  const bool p2plane = opts.mode == RST_P2PLANE;
  if (opts.mode != RST_P2POINT_REF && opts.mode != RST_P2PLANE) return RST_E_ARG;
  if (!p2plane && opts.sum_mode != RST_SUM_FP64) return RST_E_ARG;  // no shard decomposition
  if (!tgt->has_bvh || tgt->m < 1 || tgt->m > kPosMask) return RST_E_ARG;
  if (p2plane && !tgt->nrm) return RST_E_STATE;
  const int64_t n = src->m;
  *nv = p2plane ? kNP2Plane : kNP2Point;
  hipStream_t st = ctx->stream;
  const int nblk = blocks_for(n);
  if (2 * sizeof(int) * ((size_t)nblk + 1) > (size_t)96 * 1024) return RST_E_ARG;
  const int RS = p2plane ? P2PlaneAcc::RS : P2PointAcc::RS;
  const int fb_grid = fb_grid_size();
  double* slab = nullptr;
  RST_CHECK(ctx_slab(ctx, sizeof(double) * ((size_t)nblk * RS + (size_t)kFbBlocks * RS + 64), &slab));
  double* slab2 = slab + (size_t)nblk * RS;
  double* totals = slab2 + (size_t)kFbBlocks * RS;
  void* w = nullptr;
  const size_t np = (size_t)std::max<int64_t>(n, 1), nq = (size_t)nblk * kBS;
  RST_CHECK(ctx_workspace(ctx, sizeof(float4) * np * 2 + sizeof(int32_t) * (2 * nq + 4 * nblk + 192), &w));
  float4* cert = (float4*)w;
  float4* nnq = cert + np;
  int32_t* qbuf = (int32_t*)(cert + 2 * np);
  int32_t* qcnt = qbuf + 2 * nq;
  RST_HIP(hipMemsetAsync(nnq, 0xff, sizeof(float4) * np, st));
  InitArgs ia;
  memcpy(ia.pose, pose, sizeof(ia.pose));
  ia.mu0 = mu;
  ia.need_centroid = 0;
  ia.chain = 0;
  ia.n = n;
  RST_HIP(hipMemsetAsync(&ctx->d_state->guard, 0, sizeof(int32_t), st));
  k_init_state<<<1, kBS, 0, st>>>(slab, 0, nullptr, ia, ctx->d_state);
  float* dsm = (float*)(totals + 48);
  RST_HIP(hipMemcpyAsync(dsm, smean, sizeof(float) * 3, hipMemcpyHostToDevice, st));
  k_debug_state<<<1, 64, 0, st>>>(ctx->d_state, dsm, mu, iter);
  AccArgs aa;
  aa.corr = nullptr;
  aa.full_from = 0;
  aa.pix_half = aa.row_half = 0.f;
  aa.nrm = tgt->nrm;
  aa.pmu = opts.p2plane_mu;
  aa.max_d2 = opts.p2plane_max_dist > 0 ? opts.p2plane_max_dist * opts.p2plane_max_dist : FLT_MAX;
  aa.pos0 = tgt->pos0;
  const IcpParams prm = make_params(opts, n, n);
  const BvhView bv = view_of(tgt);
  const AdjView av = adj_of(tgt);
  const size_t fb_lds = 2 * sizeof(int) * ((size_t)nblk + 1);
  auto pass = [&](auto tag) {
    using Acc = typename decltype(tag)::type;
    if (n > 0) {
      k_icp_nn<Acc><<<nblk, kBS, 0, st>>>(bv, av, tgt->pix, aa, src->pts, n, ctx->d_state, nnq, cert, qbuf,
                                          qcnt, slab);
      if constexpr (Acc::kPubPrefix) k_queue_prefix<<<1, kBS, 0, st>>>(qcnt, nblk, ctx->d_state);
      k_icp_fb<Acc><<<fb_grid, kBS, fb_lds, st>>>(bv, av, tgt->pix, aa, src->pts, ctx->d_state, nnq, cert,
                                                   qbuf, qcnt, nblk, prm.lane_min, slab, slab2, n);
      k_reduce_solve<Acc><<<1, kRedBS, 0, st>>>(slab, 0, slab2, fb_grid, prm, ctx->d_state, totals);
    } else {
      (void)hipMemsetAsync(totals, 0, sizeof(double) * Acc::NV, st);
    }
  };
  if (p2plane)
    pass(AccTag<P2PlaneAcc>{});
  else
    pass(AccTag<P2PointAcc>{});
  RST_HIP(hipGetLastError());
  RST_HIP(hipMemcpyAsync(out, totals, sizeof(double) * *nv, hipMemcpyDeviceToHost, st));
  RST_HIP(hipMemcpyAsync(ctx->h_state, ctx->d_state, sizeof(IcpState), hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  if (ctx->h_state->guard) {
    set_last_error(hipErrorIllegalAddress, "ICP index guard (partials)", __FILE__, __LINE__);
    return RST_E_HIP;
  }
  return RST_OK;
}

int icp_debug_solve(rst_ctx* ctx, const rst_icp_opts* opts_in, int64_t n_total,
                    const double* totals, const float smean[3], float pose_inout[16],
                    float* mu_inout, int32_t* iter_inout) {
  if (!ctx || !totals || !smean || !pose_inout || !mu_inout || !iter_inout) return RST_E_ARG;
  rst_icp_opts opts;
  if (opts_in)
    opts = *opts_in;
  else
    rst_icp_opts_default(&opts);
  const bool p2plane = opts.mode == RST_P2PLANE;
  if (opts.mode != RST_P2POINT_REF && opts.mode != RST_P2PLANE) return RST_E_ARG;
  const int nv = p2plane ? kNP2Plane : kNP2Point;
  hipStream_t st = ctx->stream;
  double* buf = nullptr;
  RST_CHECK(ctx_slab(ctx, sizeof(double) * 64, &buf));
  RST_HIP(hipMemcpyAsync(buf, totals, sizeof(double) * nv, hipMemcpyHostToDevice, st));
  float* dsm = (float*)(buf + 48);
  RST_HIP(hipMemcpyAsync(dsm, smean, sizeof(float) * 3, hipMemcpyHostToDevice, st));
  InitArgs ia;
  memcpy(ia.pose, pose_inout, sizeof(ia.pose));
  ia.mu0 = *mu_inout;
  ia.need_centroid = 0;
  ia.chain = 0;
  ia.n = n_total;
  RST_HIP(hipMemsetAsync(&ctx->d_state->guard, 0, sizeof(int32_t), st));
  k_init_state<<<1, kBS, 0, st>>>(buf, 0, nullptr, ia, ctx->d_state);
  k_debug_state<<<1, 64, 0, st>>>(ctx->d_state, dsm, *mu_inout, *iter_inout);
  const IcpParams prm = make_params(opts, n_total, n_total);
  if (p2plane)
    k_solve_only<P2PlaneAcc><<<1, 64, 0, st>>>(buf, prm, ctx->d_state);
  else
    k_solve_only<P2PointAcc><<<1, 64, 0, st>>>(buf, prm, ctx->d_state);
  RST_HIP(hipGetLastError());
  RST_HIP(hipMemcpyAsync(ctx->h_state, ctx->d_state, sizeof(IcpState), hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  const IcpState& h = *ctx->h_state;
  for (int c = 0; c < 3; ++c) {
    for (int r = 0; r < 3; ++r) pose_inout[c * 4 + r] = h.R[c * 3 + r];
    pose_inout[c * 4 + 3] = 0.f;
  }
  for (int r = 0; r < 3; ++r) pose_inout[12 + r] = h.t[r];
  pose_inout[15] = 1.f;
  *mu_inout = h.mu;
  *iter_inout = h.iter;
  return RST_OK;
}

int icp_align_prepared(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
                       const rst_icp_opts* opts, float pose_inout[16], float* mean_cost,
                       int32_t* iters_run, rst_comm* comm) {
  const int s = icp_launch(ctx, src, tgt, opts, pose_inout, comm);
  if (s != RST_OK) return s;  // error, or the early false with the pose untouched
  return icp_finish(ctx, pose_inout, mean_cost, iters_run);
}

}  // namespace rst
