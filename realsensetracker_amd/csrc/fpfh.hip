// fpfh.hip -- the FPFH global initialisation of the align app (SURVEY.md §8f
// row f3): ComputeFpfh (fpfh.cpp:20-100,114-165,248-262) and ComputeMatches
// (fpfh.cpp:285-300) on MI355X; the caller's PruneMatchesLowe + SolveKabsch
// (rs_align_app.cpp:177-217, 286-295) run on these outputs.
//
//   k_spfh   one point per lane: radius search (the index's stackless walk,
//            every node within r^2 of the query), for each neighbour the
//            PFH triple (ComputePfh :20-64) binned into 3 x 11 counts held
//            in the lane's LDS row; the reference adds dhist = 1 / (|nbrs| -
//            1) per hit, so each bin is that float sum repeated count times
//            (exact, order-free);
//   k_fpfh   one point per lane: radius search again, feat += (1 / dist) *
//            spfh[nbr] over the neighbours but itself (33 registers), each
//            11-bin histogram scaled to sum 1 (:148-163);
//   k_match  one source feature per lane, all target features streamed
//            (wave-uniform addresses: broadcast loads), exact 1- or 2-NN in
//            33-D: nanoflann metric_L2's distance (four dimensions per
//            partial sum) and the (d2, index) order of the 1-NN kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "rst_bvh.hpp"
#include "rst_device.hpp"
#include "rst_internal.hpp"

namespace rst {
namespace {

constexpr int kBS = 128;
constexpr int kBins = 11;
constexpr int kF = 3 * kBins;

// ComputePfh (fpfh.cpp:20-64), kSymmetricPfh.  Vector3f dot / norm in
// Eigen's unrolled redux order, x0 + (x1 + x2) (redux_novec_unroller splits a
// length-3 sum 1 + 2; the same order as the oracle's mv_row).  False (f zeroed) when the
// points coincide or |u . d| >= 1
__device__ __forceinline__ bool pfh(float p1x, float p1y, float p1z, float n1x, float n1y,
                                    float n1z, float p2x, float p2y, float p2z, float n2x,
                                    float n2y, float n2z, float& f0, float& f1, float& f2) {
  float dx = p2x - p1x, dy = p2y - p1y, dz = p2z - p1z;
  const float distance = sqrtf(dx * dx + (dy * dy + dz * dz));
  if (distance == 0.0f) return false;
  const float id = 1.0f / distance;
  dx = dx * id;
  dy = dy * id;
  dz = dz * id;
  const float n1_d = n1x * dx + (n1y * dy + n1z * dz);
  const float n2_d = n2x * dx + (n2y * dy + n2z * dz);
  float u_d, nt_d;
  if (fabsf(n1_d) < fabsf(n2_d)) {
    u_d = -n2_d;
    nt_d = -n1_d;
  } else {
    u_d = n1_d;
    nt_d = n2_d;
  }
  if (fabsf(u_d) >= 1.0f) return false;
  const float v_norm = sqrtf(1.0f - u_d * u_d);
  const float n1n2 = n1x * n2x + (n1y * n2y + n1z * n2z);
  f0 = atan2f(nt_d - n1n2 * u_d, n1n2 * v_norm);
  const float cx = n1y * n2z - n1z * n2y, cy = n1z * n2x - n1x * n2z, cz = n1x * n2y - n1y * n2x;
  f1 = (dx * cx + (dy * cy + dz * cz)) / v_norm;
  f2 = u_d;
  return true;
}

// (:86-90) floor(kNumBins * (f * scale + 0.5)) in double, clamped
__device__ __forceinline__ int pfh_bin(float f, float scale) {
  const int raw = (int)floor((double)kBins * ((double)(f * scale) + 0.5));
  return max(0, min(kBins - 1, raw));
}

struct SpfhVisitor {
  float r2;
  int self;
  float px, py, pz, nx, ny, nz;
  const float4* __restrict__ pts;
  const float4* __restrict__ nrm;
  int* hist;  // this lane's LDS row, kF counts
  int cnt;    // |nbrs| (self included, as the reference's radius search)
  __device__ float bound() const { return r2; }
  __device__ void offer(float d2, int id, int pos) {
    (void)id;
    if (!(d2 < r2)) return;  // nanoflann RadiusResultSet: dist < radius
    ++cnt;
    if (pos == self) return;
    const float4 q = pts[pos], m = nrm[pos];
    float f0, f1, f2;
    if (!pfh(px, py, pz, nx, ny, nz, q.x, q.y, q.z, m.x, m.y, m.z, f0, f1, f2)) return;
    const float s0 = (float)(1.0 / (2.0 * M_PI));  // scale (:76)
    hist[pfh_bin(f0, s0)] += 1;
    hist[kBins + pfh_bin(f1, 0.5f)] += 1;
    hist[2 * kBins + pfh_bin(f2, 0.5f)] += 1;
  }
};

__global__ __launch_bounds__(kBS) void k_spfh(BvhView bv, const float4* __restrict__ nrm, float r2,
                                              float* __restrict__ spfh) {
  __shared__ int hist[kBS * kF];
  const int64_t p = blockIdx.x * (int64_t)kBS + threadIdx.x;
  int* h = hist + threadIdx.x * kF;
  for (int b = 0; b < kF; ++b) h[b] = 0;
  if (p >= bv.m) return;  // no block-wide sync below
  const float4 q = bv.pts[p], n = nrm[p];
  SpfhVisitor v{r2, (int)p, q.x, q.y, q.z, n.x, n.y, n.z, bv.pts, nrm, h, 0};
  descend(bv, 1, q.x, q.y, q.z, v);
  const float dhist = 1.0f / (float)(v.cnt - 1);  // (:78) 1.0f / (nbrs.size() - 1)
  float* out = spfh + p * kF;
  for (int b = 0; b < kF; ++b) {
    float s = 0.0f;
    for (int c = 0; c < h[b]; ++c) s = s + dhist;  // += dhist per hit (:91)
    out[b] = s;
  }
}

struct FpfhVisitor {
  float r2;
  int self;
  const float* __restrict__ spfh;
  float acc[kF];
  __device__ float bound() const { return r2; }
  __device__ void offer(float d2, int id, int pos) {
    (void)id;
    if (!(d2 < r2) || pos == self) return;  // skip self (:145-148)
    const float w = 1.0F / sqrtf(d2);        // (:150-151)
    const float* s = spfh + (int64_t)pos * kF;
#pragma unroll
    for (int b = 0; b < kF; ++b) acc[b] = acc[b] + w * s[b];
  }
};

__global__ __launch_bounds__(kBS) void k_fpfh(BvhView bv, const float* __restrict__ spfh, float r2,
                                              float* __restrict__ out) {
  const int64_t p = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (p >= bv.m) return;
  const float4 q = bv.pts[p];
  FpfhVisitor v;
  v.r2 = r2;
  v.self = (int)p;
  v.spfh = spfh;
#pragma unroll
  for (int b = 0; b < kF; ++b) v.acc[b] = 0.0f;
  descend(bv, 1, q.x, q.y, q.z, v);
  // (:155-162) each histogram to sum 1
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float s = 0.0f;
#pragma unroll
    for (int b = 0; b < kBins; ++b) s = s + v.acc[k * kBins + b];
    if (s > 0) {
      const float inv = 1.0f / s;
#pragma unroll
      for (int b = 0; b < kBins; ++b) v.acc[k * kBins + b] = v.acc[k * kBins + b] * inv;
    }
  }
  float* o = out + (int64_t)f2i(q.w) * kF;
#pragma unroll
  for (int b = 0; b < kF; ++b) o[b] = v.acc[b];
}

// nanoflann metric_L2 (L2_Adaptor::evalMetric) in 33-D: four dimensions per
// partial sum, then the last one (oracle orc_feat_d2)
__device__ __forceinline__ float feat_d2(const float (&a)[kF], const float* __restrict__ b) {
  float r = 0.0f;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const float d0 = a[4 * g] - b[4 * g], d1 = a[4 * g + 1] - b[4 * g + 1];
    const float d2 = a[4 * g + 2] - b[4 * g + 2], d3 = a[4 * g + 3] - b[4 * g + 3];
    r = r + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
  }
  const float d = a[32] - b[32];
  return r + d * d;
}

__global__ __launch_bounds__(256) void k_match(const float* __restrict__ src, int64_t n,
                                               const float* __restrict__ dst, int64_t m, int k,
                                               int32_t* __restrict__ idx,
                                               float* __restrict__ d2out) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  const bool act = i < n;
  float a[kF];
#pragma unroll
  for (int b = 0; b < kF; ++b) a[b] = act ? src[i * kF + b] : 0.0f;
  float b0 = FLT_MAX, b1 = FLT_MAX;
  int i0 = 0, i1 = 0;
  bool h0 = false, h1 = false;
  for (int64_t j = 0; j < m; ++j) {  // wave-uniform: every lane reads dst row j
    const float d = feat_d2(a, dst + j * kF);
    const int jj = (int)j;
    if (!h0 || lex_less(d, jj, b0, i0)) {
      b1 = b0;
      i1 = i0;
      h1 = h0;
      b0 = d;
      i0 = jj;
      h0 = true;
    } else if (!h1 || lex_less(d, jj, b1, i1)) {
      b1 = d;
      i1 = jj;
      h1 = true;
    }
  }
  if (!act) return;
  idx[i * k] = i0;
  if (d2out) d2out[i * k] = b0;
  if (k > 1) {
    idx[i * k + 1] = h1 ? i1 : 0;
    if (d2out) d2out[i * k + 1] = h1 ? b1 : FLT_MAX;
  }
}

inline int blocks_for(int64_t n, int per) {
  return (int)std::max<int64_t>(1, (n + per - 1) / per);
}

}  // namespace
}  // namespace rst

using namespace rst;

extern "C" {

int rst_compute_fpfh(rst_ctx* ctx, const float* xyz, int64_t n, const float viewpoint[3],
                     int normal_k, float radius, float* fpfh_out) {
  if (!ctx || !viewpoint || n < 0 || (n > 0 && (!xyz || !fpfh_out)) ||
      (normal_k != 8 && normal_k != 16 && normal_k != 32) || !(radius > 0.f) ||
      (n > 0 && n < normal_k))
    return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  if (n == 0) return RST_OK;
  hipStream_t st = ctx->stream;
  float* d = nullptr;
  size_t cd = 0;
  RST_CHECK(ctx_alloc(ctx, sizeof(float) * 3 * n, (void**)&d, &cd));
  rst_target* t = nullptr;
  float *spfh = nullptr, *out = nullptr;
  size_t cs = 0, co = 0;
  int s = hipMemcpyAsync(d, xyz, sizeof(float) * 3 * n, hipMemcpyHostToDevice, st) == hipSuccess
              ? RST_OK
              : RST_E_HIP;
  // (:248-258) the index (leaf 16), normals + orientation, then the features
  if (s >= 0) s = target_build_device(ctx, d, n, true, &t);
  if (s >= 0) s = compute_normals(ctx, t, normal_k, viewpoint);
  if (s >= 0) s = ctx_alloc(ctx, sizeof(float) * kF * n, (void**)&spfh, &cs);
  if (s >= 0) s = ctx_alloc(ctx, sizeof(float) * kF * n, (void**)&out, &co);
  if (s >= 0) {
    const BvhView bv = view_of(t);
    const float r2 = radius * radius;  // (:123) radius_sq
    k_spfh<<<blocks_for(n, kBS), kBS, 0, st>>>(bv, t->nrm, r2, spfh);
    k_fpfh<<<blocks_for(n, kBS), kBS, 0, st>>>(bv, spfh, r2, out);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(fpfh_out, out, sizeof(float) * kF * n, hipMemcpyDeviceToHost, st) !=
            hipSuccess)
      s = RST_E_HIP;
  }
  hipStreamSynchronize(st);
  if (t) rst_target_free(t);
  ctx_release(ctx, d, cd);
  if (spfh) ctx_release(ctx, spfh, cs);
  if (out) ctx_release(ctx, out, co);
  return s < 0 ? s : RST_OK;
}

int rst_compute_matches(rst_ctx* ctx, const float* src_feat, int64_t n, const float* dst_feat,
                        int64_t m, int k, int32_t* idx_out, float* d2_out) {
  if (!ctx || n < 0 || m < 1 || k < 1 || k > 2 || (n > 0 && (!src_feat || !idx_out)) ||
      !dst_feat)
    return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  if (n == 0) return RST_OK;
  hipStream_t st = ctx->stream;
  float *ds = nullptr, *dd = nullptr, *dd2 = nullptr;
  int32_t* di = nullptr;
  size_t c1 = 0, c2 = 0, c3 = 0, c4 = 0;
  RST_CHECK(ctx_alloc(ctx, sizeof(float) * kF * n, (void**)&ds, &c1));
  int s = ctx_alloc(ctx, sizeof(float) * kF * m, (void**)&dd, &c2);
  if (s >= 0) s = ctx_alloc(ctx, sizeof(int32_t) * k * n, (void**)&di, &c3);
  if (s >= 0) s = ctx_alloc(ctx, sizeof(float) * k * n, (void**)&dd2, &c4);
  if (s >= 0 &&
      (hipMemcpyAsync(ds, src_feat, sizeof(float) * kF * n, hipMemcpyHostToDevice, st) !=
           hipSuccess ||
       hipMemcpyAsync(dd, dst_feat, sizeof(float) * kF * m, hipMemcpyHostToDevice, st) !=
           hipSuccess))
    s = RST_E_HIP;
  if (s >= 0) {
    k_match<<<blocks_for(n, 256), 256, 0, st>>>(ds, n, dd, m, k, di, dd2);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(idx_out, di, sizeof(int32_t) * k * n, hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        (d2_out && hipMemcpyAsync(d2_out, dd2, sizeof(float) * k * n, hipMemcpyDeviceToHost,
                                  st) != hipSuccess))
      s = RST_E_HIP;
  }
  hipStreamSynchronize(st);
  ctx_release(ctx, ds, c1);
  if (dd) ctx_release(ctx, dd, c2);
  if (di) ctx_release(ctx, di, c3);
  if (dd2) ctx_release(ctx, dd2, c4);
  return s < 0 ? s : RST_OK;
}

}  // extern "C"
