// gicp.hip -- the align module's second registration path (SURVEY.md §8f
// row f2): GICP ComputeAlignment (align_gicp.cpp:41-163) with its
// ComputeCovariances (point_cloud_utils.cpp:100-161), on MI355X.
//
//   k_covariances      one point per lane: exact 33-NN in its own cloud's
//                      index (self first, dropped), fp32 centroid and outer
//                      products in result order, / 31 (use_gicp: the
//                      I - 0.99 u3 u3^T regularisation, :139-155);
//   k_gicp_eval        one correspondence per lane, fp64: C = S_d + R S_s R^T,
//                      its inverse square root through a 3x3 Jacobi
//                      eigen-decomposition, residual r = C^-1/2 (R s + t - d)
//                      (gicp_cost.hpp:40-73), Huber(0.5) (align_gicp.cpp:70)
//                      as Ceres' corrector weights it (rho'' <= 0: J~ =
//                      sqrt(rho') J), the exact 3x6 Jacobian (rotation
//                      perturbation exp([w]x) R, including d C^-1/2 / dw),
//                      28 fp64 partial sums (H 21, g 6, cost) per block;
//   k_gicp_lm          one block: fixed-order reduction, then thread 0 runs
//                      one Levenberg-Marquardt decision (accept / reject,
//                      damping) and proposes the next candidate.
//
// Ceres' LM (DENSE_QR, its own trust-region schedule) is restated as the
// build's LM (oracle/rst_oracle.c orc_gicp_solve, the same decisions): the
// optimum is the cost's, the path to it is not Ceres'.  The outer loop of
// the three-argument ComputeAlignment (16 x {exact 1-NN of estimate * src;
// LM from estimate}) stays on the device; one host sync at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "rst_bvh.hpp"
#include "rst_device.hpp"
#include "rst_internal.hpp"

namespace rst {
namespace {

constexpr int kBS = 256;
constexpr int kRedBS = 1024;
constexpr int kNV = 28;  // H upper (21), g (6), cost
constexpr int kRS = 32;  // slab row stride
constexpr int kKnn = 33;
// stop once an accepted step lowers the cost by less than this fraction:
// Ceres' default Solver::Options::function_tolerance (the reference's
// GetOptions(), align_gicp.cpp:13-37, sets none)
constexpr double kGicpFtol = 1e-6;

struct GicpState {
  double R[9], t[3];     // accepted pose (row-major R)
  double Rc[9], tc[3];   // candidate under evaluation
  double H[36], g[6];    // accepted normal equations
  double F;              // accepted cost
  double lambda;
  int iters;             // evaluations done
  int done;
  int max_iter;
  int pad;
  float est[16];         // outer-loop estimate (col-major float pose)
};

// ---- ComputeCovariances ------------------------------------------------------------
// (:121-158) the covariance of one point from its 33 nearest (sorted
// positions in result order, < 0: a slot the search could not fill, which
// the reference's out-parameters leave at index 0): fp32 centroid of results
// 1..32, fp32 outer-product sums, then the GICP plane form or / 31
__device__ __forceinline__ void cov_from_results(const BvhView& bv, int32_t pos0, int use_gicp,
                                                 const int* pos, int orig, float* covs) {
  float cx = 0.f, cy = 0.f, cz = 0.f;
#pragma unroll
  for (int j = 1; j < kKnn; ++j) {
    const float4 o = bv.pts[pos[j] >= 0 ? pos[j] : pos0];
    cx = cx + o.x;
    cy = cy + o.y;
    cz = cz + o.z;
  }
  cx = cx / 32.0f;
  cy = cy / 32.0f;
  cz = cz / 32.0f;
  float c[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) c[k] = 0.f;
#pragma unroll
  for (int j = 1; j < kKnn; ++j) {  // (:130-135)
    const float4 o = bv.pts[pos[j] >= 0 ? pos[j] : pos0];
    const float d[3] = {o.x - cx, o.y - cy, o.z - cz};
#pragma unroll
    for (int cc = 0; cc < 3; ++cc)
#pragma unroll
      for (int r = 0; r < 3; ++r) c[cc * 3 + r] = c[cc * 3 + r] + d[r] * d[cc];
  }
  float* out = covs + 9 * (int64_t)orig;
  if (use_gicp) {  // (:139-155): U diag(1, 1, 1e-2) U^T = I - 0.99 u3 u3^T
    double a[9], U[9], S[3], V[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) a[k] = c[k];
    svd3_jacobi(a, U, S, V);
    const int kmin = (S[0] <= S[1] && S[0] <= S[2]) ? 0 : (S[1] <= S[2] ? 1 : 2);
    double u[3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
      u[r] = kmin == 0 ? RST_M3(U, r, 0) : (kmin == 1 ? RST_M3(U, r, 1) : RST_M3(U, r, 2));
#pragma unroll
    for (int cc = 0; cc < 3; ++cc)
#pragma unroll
      for (int r = 0; r < 3; ++r)
        out[cc * 3 + r] = (float)((r == cc ? 1.0 : 0.0) - (1.0 - 1e-2) * u[r] * u[cc]);
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) out[k] = c[k] / 31.0f;  // (:158)
  }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = ((uint64_t)(uint32_t)__shfl_xor((int)(x >> 32), o, 64) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)x, o, 64);
    x = y < x ? y : x;
  }
  return x;
}

// (d2, original index) as one ordered key: d2 >= 0 (or +inf), so its bits
// order as the float; the lexicographic order of BestK / Best1
__device__ __forceinline__ uint64_t nn_key(float d2, int id) {
  return ((uint64_t)(uint32_t)f2i(d2) << 32) | (uint32_t)id;
}

// Small clouds (GICP's voxel-downsampled frames, a few thousand points):
// one wavefront per point, every target point's key staged in LDS (the
// lanes stride the cloud), then the 33 smallest keys extracted in order,
// one wave minimum per result -- the same exact 33-NN in the same order as
// the per-lane BVH search (k_covariances), on a wavefront per point instead
// of a lane: the BVH kernel leaves a 4k-point cloud on 18 of 256 CUs.
constexpr int kCovWaveMax = 8000;  // LDS keys per wavefront (< 64 KB with the result slots)
__global__ __launch_bounds__(kWave) void k_covariances_wave(BvhView bv, int32_t pos0,
                                                            int use_gicp,
                                                            float* __restrict__ covs) {
  extern __shared__ uint64_t keys[];  // [m]
  __shared__ int res[kKnn];
  const int p = blockIdx.x;  // sorted position of the point
  const int lane = threadIdx.x;
  const int m = bv.m;
  const float4 q = bv.pts[p];
  for (int j = lane; j < m; j += kWave) {
    const float4 t = bv.pts[j];
    keys[j] = nn_key(d2_ref(q.x, q.y, q.z, t.x, t.y, t.z), f2i(t.w));
  }
  __syncthreads();  // (one wavefront per block)
  uint64_t last = 0;
  for (int k = 0; k < kKnn; ++k) {
    uint64_t best = ~0ull;
    int bj = -1;
    for (int j = lane; j < m; j += kWave) {
      const uint64_t x = keys[j];
      if ((k == 0 || x > last) && x < best) {
        best = x;
        bj = j;
      }
    }
    const uint64_t w = wave_min_u64(best);
    const uint64_t bm = __ballot(bj >= 0 && best == w);
    const int src = bm ? __ffsll((long long)bm) - 1 : 0;
    const int wj = __shfl(bj, src, kWave);
    if (lane == 0) res[k] = bm ? wj : -1;
    last = w;
  }
  __syncthreads();  // (one wavefront per block)
  if (lane == 0) {
    int pos[kKnn];
#pragma unroll
    for (int k = 0; k < kKnn; ++k) pos[k] = res[k];
    cov_from_results(bv, pos0, use_gicp, pos, f2i(q.w), covs);
  }
}

// A cloud as the brute-force kernels read it: (x, y, z, index bits) in input
// order (sorted position = original index, so pos0 = 0)
__global__ __launch_bounds__(kBS) void k_pack4(const float* __restrict__ xyz, int64_t n,
                                               float4* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i < n) out[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], i2f((int)i));
}

// Exact NN of each query over a small cloud, one wavefront per query (the
// lanes stride the cloud, a wave minimum of the (d2, index) keys): GICP's
// per-round correspondences, where the BVH kernel's one lane per query
// leaves the GPU idle.
__global__ __launch_bounds__(kBS) void k_query_nn_wave(BvhView bv, const float* __restrict__ q,
                                                       int64_t nq, int32_t* __restrict__ idx,
                                                       float* __restrict__ d2) {
  const int64_t i = (int64_t)blockIdx.x * (kBS / kWave) + threadIdx.x / kWave;
  if (i >= nq) return;  // (uniform per wave)
  const int lane = threadIdx.x & (kWave - 1);
  const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
  uint64_t best = ~0ull;
  for (int j = lane; j < bv.m; j += kWave) {
    const float4 t = bv.pts[j];
    const uint64_t x = nn_key(d2_ref(qx, qy, qz, t.x, t.y, t.z), f2i(t.w));
    best = x < best ? x : best;
  }
  best = wave_min_u64(best);
  if (lane == 0) {
    idx[i] = best == ~0ull ? -1 : (int32_t)(uint32_t)best;
    d2[i] = best == ~0ull ? FLT_MAX : i2f((int)(best >> 32));
  }
}


__global__ __launch_bounds__(kBS) void k_covariances(BvhView bv, int32_t pos0, int use_gicp,
                                                     float* __restrict__ covs) {
  const int64_t p = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (p >= bv.m) return;
  const float4 q = bv.pts[p];
  BestK<kKnn> L;
  L.init();
  search(bv, (int)p, q.x, q.y, q.z, L);
  cov_from_results(bv, pos0, use_gicp, L.pos, f2i(q.w), covs);
}

// ---- per-correspondence evaluation ---------------------------------------------------
// symmetric 3x3 eigen-decomposition, cyclic Jacobi (the oracle's
// gicp_sym_eig3); all indices static after unrolling
__device__ __forceinline__ void sym_eig3(double (&a)[3][3], double (&v)[3][3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) v[r][c] = r == c ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; ++sweep) {
    const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    const double dg = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
    if (!(off > 1e-32 * dg)) break;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int p = k == 2 ? 1 : 0, q = k == 0 ? 1 : 2;
      const double apq = a[p][q];
      if (apq != 0.0) {
        const double th = (a[q][q] - a[p][p]) / (2.0 * apq);
        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const double arp = a[r][p], arq = a[r][q];
          a[r][p] = c * arp - s * arq;
          a[r][q] = s * arp + c * arq;
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const double apr = a[p][r], aqr = a[q][r];
          a[p][r] = c * apr - s * aqr;
          a[q][r] = s * apr + c * aqr;
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const double vrp = v[r][p], vrq = v[r][q];
          v[r][p] = c * vrp - s * vrq;
          v[r][q] = s * vrp + c * vrq;
        }
      }
    }
  }
}

__global__ __launch_bounds__(kBS) void k_gicp_eval(const float* __restrict__ src, int64_t n,
                                                   const float* __restrict__ dst,
                                                   const float* __restrict__ scov,
                                                   const float* __restrict__ dcov,
                                                   const int32_t* __restrict__ idx,
                                                   const GicpState* __restrict__ st,
                                                   double* __restrict__ slab) {
  __shared__ double lds[(kBS / kWave) * kNV];
  if (st->done) return;  // uniform
  double v[kNV];
#pragma unroll
  for (int k = 0; k < kNV; ++k) v[k] = 0.0;
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i < n) {
    double R[3][3], t[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) R[r][c] = st->Rc[3 * r + c];
      t[r] = st->tc[r];
    }
    const int64_t j = idx[i];
    double Ss[3][3], Sd[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        Ss[r][c] = scov[9 * i + 3 * c + r];  // col-major (Eigen)
        Sd[r][c] = dcov[9 * j + 3 * c + r];
      }
    double RS[3][3], A[3][3], C[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) s += R[r][k] * Ss[k][c];
        RS[r][c] = s;
      }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) s += RS[r][k] * R[c][k];
        A[r][c] = s;
        C[r][c] = Sd[r][c] + s;
      }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = r + 1; c < 3; ++c) {
        const double m = 0.5 * (C[r][c] + C[c][r]);
        C[r][c] = m;
        C[c][r] = m;
      }
    double V[3][3];
    sym_eig3(C, V);
    double lam[3], is[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      lam[k] = C[k][k] > 1e-30 ? C[k][k] : 1e-30;
      is[k] = 1.0 / sqrt(lam[k]);
    }
    double M[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) s += V[r][k] * is[k] * V[c][k];
        M[r][c] = s;
      }
    const double sx = src[3 * i], sy = src[3 * i + 1], sz = src[3 * i + 2];
    double Rs[3], dl[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      Rs[r] = R[r][0] * sx + R[r][1] * sy + R[r][2] * sz;
      dl[r] = Rs[r] + t[r] - (double)dst[3 * j + r];
    }
    double res[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) res[r] = M[r][0] * dl[0] + M[r][1] * dl[1] + M[r][2] * dl[2];
    const double s2 = res[0] * res[0] + res[1] * res[1] + res[2] * res[2];
    const double rho = s2 <= 0.25 ? s2 : sqrt(s2) - 0.25;
    const double rho1 = s2 <= 0.25 ? 1.0 : 0.5 / sqrt(s2);
    double W[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b)
        W[a][b] = fabs(lam[a] - lam[b]) > 1e-12 * (lam[a] + lam[b])
                      ? (is[a] - is[b]) / (lam[a] - lam[b])
                      : -0.5 * is[a] / lam[a];
    double J[3][6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      // E = G_k A - A G_k, G_k = [e_k]x
      double E[3][3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          // (G A)(r,c) = sum_q G(r,q) A(q,c); G(r,q) = -eps(k,r,q)
          double ga = 0, ag = 0;
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const double grq = (k == 0) ? ((r == 1 && q == 2) ? -1.0 : ((r == 2 && q == 1) ? 1.0 : 0.0))
                             : (k == 1) ? ((r == 0 && q == 2) ? 1.0 : ((r == 2 && q == 0) ? -1.0 : 0.0))
                                        : ((r == 0 && q == 1) ? -1.0 : ((r == 1 && q == 0) ? 1.0 : 0.0));
            const double gqc = (k == 0) ? ((q == 1 && c == 2) ? -1.0 : ((q == 2 && c == 1) ? 1.0 : 0.0))
                             : (k == 1) ? ((q == 0 && c == 2) ? 1.0 : ((q == 2 && c == 0) ? -1.0 : 0.0))
                                        : ((q == 0 && c == 1) ? -1.0 : ((q == 1 && c == 0) ? 1.0 : 0.0));
            ga += grq * A[q][c];
            ag += A[r][q] * gqc;
          }
          E[r][c] = ga - ag;
        }
      double B[3][3];
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          double s = 0;
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) s += V[r][a] * E[r][c] * V[c][b];
          B[a][b] = s * W[a][b];
        }
      double T[3][3], dM[3][3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          double s = 0;
#pragma unroll
          for (int a = 0; a < 3; ++a) s += V[r][a] * B[a][b];
          T[r][b] = s;
        }
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          double s = 0;
#pragma unroll
          for (int b = 0; b < 3; ++b) s += T[r][b] * V[c][b];
          dM[r][c] = s;
        }
      // d(delta)/dw_k = e_k x (R s)
      const double ex0 = k == 0 ? 0.0 : (k == 1 ? Rs[2] : -Rs[1]);
      const double ex1 = k == 0 ? -Rs[2] : (k == 1 ? 0.0 : Rs[0]);
      const double ex2 = k == 0 ? Rs[1] : (k == 1 ? -Rs[0] : 0.0);
#pragma unroll
      for (int r = 0; r < 3; ++r)
        J[r][k] = dM[r][0] * dl[0] + dM[r][1] * dl[1] + dM[r][2] * dl[2] + M[r][0] * ex0 +
                  M[r][1] * ex1 + M[r][2] * ex2;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) J[r][3 + c] = M[r][c];
    int h = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = a; b < 6; ++b) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < 3; ++r) s += J[r][a] * J[r][b];
        v[h++] = rho1 * s;
      }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      double s = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) s += J[r][a] * res[r];
      v[21 + a] = rho1 * s;
    }
    v[27] = 0.5 * rho;
  }
  block_sum_to_slab<kNV, kBS>(v, lds, slab + (int64_t)blockIdx.x * kRS);
}

// ---- LM decision (one block) ---------------------------------------------------------
__device__ void rodrigues(const double w[3], double (&E)[3][3]) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const double th = sqrt(th2);
  double a, b;
  if (th < 1e-8) {
    a = 1.0 - th2 / 6.0;
    b = 0.5 - th2 / 24.0;
  } else {
    a = sin(th) / th;
    b = (1.0 - cos(th)) / th2;
  }
  const double K[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double kk = 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) kk += K[r][q] * K[q][c];
      E[r][c] = (r == c ? 1.0 : 0.0) + a * K[r][c] + b * kk;
    }
}

// (H + lambda diag(H)) x = -g, Cholesky; false when not positive definite
__device__ bool lm_step(const double (&H)[6][6], const double (&g)[6], double lambda,
                        double (&x)[6]) {
  double L[6][6];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) L[a][b] = H[a][b] + (a == b ? lambda * H[a][a] : 0.0);
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double s = L[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
    if (!(s > 0)) return false;
    L[j][j] = sqrt(s);
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double u = L[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) u -= L[i][k] * L[j][k];
      L[i][j] = u / L[j][j];
    }
  }
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = -g[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  return true;
}

__global__ __launch_bounds__(kRedBS) void k_gicp_lm(const double* __restrict__ slab, int rows,
                                                    GicpState* __restrict__ st) {
  constexpr int PER = kRedBS / kRS;
  __shared__ double red[kRedBS];
  __shared__ double tot[kRS];
  if (st->done) return;
  const int t = threadIdx.x, col = t % kRS;
  double acc = 0.0;
  for (int r = t / kRS; r < rows; r += PER) acc += slab[(int64_t)r * kRS + col];
  red[t] = acc;
  __syncthreads();
  if (t < kRS) {
    double x = 0.0;
    for (int j = 0; j < PER; ++j) x += red[j * kRS + t];
    tot[t] = x;
  }
  __syncthreads();
  if (t != 0) return;
  GicpState& s = *st;
  const double F2 = tot[27];
  const int it = s.iters++;
  bool accept;
  if (it == 0) {
    accept = true;  // the seed's evaluation
  } else {
    accept = F2 < s.F;
  }
  if (accept) {
    const double drop = it == 0 ? 1.0 : (s.F - F2) / (s.F > 0 ? s.F : 1.0);
    int h = 0;
    for (int a = 0; a < 6; ++a)
      for (int b = a; b < 6; ++b) {
        s.H[6 * a + b] = tot[h];
        s.H[6 * b + a] = tot[h];
        ++h;
      }
    for (int a = 0; a < 6; ++a) s.g[a] = tot[21 + a];
    for (int k = 0; k < 9; ++k) s.R[k] = s.Rc[k];
    for (int k = 0; k < 3; ++k) s.t[k] = s.tc[k];
    s.F = F2;
    if (it > 0) {
      s.lambda = s.lambda / 3.0 > 1e-12 ? s.lambda / 3.0 : 1e-12;
      if (drop < kGicpFtol) {
        s.done = 1;
        return;
      }
    }
  } else {
    s.lambda *= 4.0;
    if (s.lambda > 1e10) {
      s.done = 1;
      return;
    }
  }
  if (s.iters >= s.max_iter) {
    s.done = 1;
    return;
  }
  // next candidate: retry the damping until the system is positive definite
  double H[6][6], g[6], x[6];
  for (int a = 0; a < 6; ++a) {
    g[a] = s.g[a];
    for (int b = 0; b < 6; ++b) H[a][b] = s.H[6 * a + b];
  }
  while (!lm_step(H, g, s.lambda, x)) {
    s.lambda *= 4.0;
    if (s.lambda > 1e10) {
      s.done = 1;
      return;
    }
  }
  const double nx = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3] + x[4] * x[4] +
                         x[5] * x[5]);
  if (nx < 1e-10) {
    s.done = 1;
    return;
  }
  double E[3][3];
  rodrigues(x, E);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      double v = 0;
      for (int q = 0; q < 3; ++q) v += E[r][q] * s.R[3 * q + c];
      s.Rc[3 * r + c] = v;
    }
  for (int r = 0; r < 3; ++r) s.tc[r] = s.t[r] + x[3 + r];
}

// seed the LM from the float estimate (col-major 4x4)
__global__ void k_gicp_begin(GicpState* __restrict__ st, int max_iter) {
  GicpState& s = *st;
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) s.Rc[3 * r + c] = s.est[4 * c + r];
    s.tc[r] = s.est[12 + r];
  }
  s.F = 0.0;
  s.lambda = 1e-4;
  s.iters = 0;
  s.done = 0;
  s.max_iter = max_iter;
}

// estimate <- the LM's accepted pose
__global__ void k_gicp_end(GicpState* __restrict__ st) {
  GicpState& s = *st;
  for (int c = 0; c < 3; ++c) {
    for (int r = 0; r < 3; ++r) s.est[4 * c + r] = (float)s.R[3 * r + c];
    s.est[4 * c + 3] = 0.f;
  }
  for (int r = 0; r < 3; ++r) s.est[12 + r] = (float)s.t[r];
  s.est[15] = 1.f;
}

// estimate * src (align_icp.cpp:107's operation order), AoS
__global__ __launch_bounds__(kBS) void k_gicp_xform(const float* __restrict__ src, int64_t n,
                                                    const GicpState* __restrict__ st,
                                                    float* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  Pose3 P;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) P.r[3 * c + r] = st->est[4 * c + r];  // column-major
#pragma unroll
  for (int r = 0; r < 3; ++r) P.t[r] = st->est[12 + r];
  float x, y, z;
  xform(P, src[3 * i], src[3 * i + 1], src[3 * i + 2], x, y, z);
  out[3 * i] = x;
  out[3 * i + 1] = y;
  out[3 * i + 2] = z;
}

inline int blocks_for(int64_t n, int per = kBS) {
  return (int)std::max<int64_t>(1, (n + per - 1) / per);
}

// device buffers of one GICP problem (all context-pool allocations)
struct Bufs {
  rst_ctx* ctx = nullptr;
  void* p[12] = {};
  size_t c[12] = {};
  int k = 0;
  int get(size_t bytes, void** out) {
    const int s = ctx_alloc(ctx, std::max<size_t>(bytes, 16), &p[k], &c[k]);
    if (s >= 0) *out = p[k++];
    return s;
  }
  ~Bufs() {
    if (ctx) hipStreamSynchronize(ctx->stream);
    for (int i = 0; i < k; ++i) ctx_release(ctx, p[i], c[i]);
  }
};

int upload(hipStream_t st, void* d, const void* h, size_t bytes) {
  RST_HIP(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
  return RST_OK;
}

// max_inner LM evaluations on (src, dst, covs, idx) from st->est; result in
// st->est.  The evaluations are enqueued kLmChunk at a time; after each
// chunk the state's `done` flag is copied to pinned host memory, and the
// host stops enqueueing once a finished chunk reports it (checked one chunk
// behind, so the device never waits for the host): a solve that converges
// after k evaluations launches about k + 2 kLmChunk of them, not max_inner
// (every launch after `done` exits at once, so the result is the same).
constexpr int kLmChunk = 4;
int lm_solve(rst_ctx* ctx, const float* ds, int64_t n, const float* dd, const float* dcs,
             const float* dcd, const int32_t* didx, GicpState* dst_state, double* slab,
             int max_inner) {
  hipStream_t st = ctx->stream;
  const int nb = blocks_for(n);
  void* pin = nullptr;
  RST_CHECK(ctx_pinned_small(ctx, 64, &pin));
  volatile int* hflag = (volatile int*)pin;
  hipEvent_t ev[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; ++k)
    if (hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) ev[k] = nullptr;
  const bool early = ev[0] && ev[1];
  k_gicp_begin<<<1, 1, 0, st>>>(dst_state, max_inner);
  int s = RST_OK;
  for (int it = 0, c = 0; it < max_inner; ++c) {
    for (int k = 0; k < kLmChunk && it < max_inner; ++k, ++it) {
      k_gicp_eval<<<nb, kBS, 0, st>>>(ds, n, dd, dcs, dcd, didx, dst_state, slab);
      k_gicp_lm<<<1, kRedBS, 0, st>>>(slab, nb, dst_state);
    }
    if (!early) continue;
    if (hipMemcpyAsync((void*)(hflag + (c & 1)), &dst_state->done, sizeof(int),
                       hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipEventRecord(ev[c & 1], st) != hipSuccess) {
      s = RST_E_HIP;
      break;
    }
    if (c >= 1) {
      if (hipEventSynchronize(ev[(c - 1) & 1]) != hipSuccess) {
        s = RST_E_HIP;
        break;
      }
      if (hflag[(c - 1) & 1]) break;  // converged: the rest would exit at once
    }
  }
  k_gicp_end<<<1, 1, 0, st>>>(dst_state);
  // (a flag copy still pending is stream-ordered before the next solve's
  // copies; the small pinned area lives as long as the context)
  for (int k = 0; k < 2; ++k)
    if (ev[k]) (void)hipEventDestroy(ev[k]);
  RST_CHECK(s);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

}  // namespace

int compute_covariances_device(rst_ctx* ctx, const rst_target* tgt, int use_gicp, float* d_covs) {
  if (!tgt->has_bvh) return RST_E_STATE;
  if (tgt->m == 0) return RST_OK;
  if (tgt->m <= kCovWaveMax)
    k_covariances_wave<<<(unsigned)tgt->m, kWave, sizeof(uint64_t) * tgt->m, ctx->stream>>>(
        view_of(tgt), tgt->pos0, use_gicp, d_covs);
  else
    k_covariances<<<blocks_for(tgt->m), kBS, 0, ctx->stream>>>(view_of(tgt), tgt->pos0, use_gicp,
                                                               d_covs);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

}  // namespace rst

using namespace rst;

extern "C" {

int rst_compute_covariances(rst_ctx* ctx, const rst_target* tgt, int use_gicp, float* covs_out) {
  if (!ctx || !tgt || !covs_out) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  if (tgt->m == 0) return RST_OK;
  Bufs b;
  b.ctx = ctx;
  float* d = nullptr;
  RST_CHECK(b.get(sizeof(float) * 9 * tgt->m, (void**)&d));
  RST_CHECK(compute_covariances_device(ctx, tgt, use_gicp, d));
  RST_HIP(hipMemcpyAsync(covs_out, d, sizeof(float) * 9 * tgt->m, hipMemcpyDeviceToHost,
                         ctx->stream));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return RST_OK;
}

int rst_gicp_solve(rst_ctx* ctx, const float* src, int64_t n, const float* dst, int64_t m,
                   const float* src_covs, const float* dst_covs, const int32_t* dst_idx,
                   const float seed[16], int max_iter, float pose_out[16], double* cost_out,
                   int32_t* iters_out) {
  if (!ctx || !src || !dst || !src_covs || !dst_covs || !dst_idx || !seed || !pose_out ||
      n < 1 || m < 1 || max_iter < 1)
    return RST_E_ARG;
  for (int64_t i = 0; i < n; ++i)
    if (dst_idx[i] < 0 || dst_idx[i] >= m) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  Bufs b;
  b.ctx = ctx;
  float *ds, *dd, *dcs, *dcd;
  int32_t* di;
  GicpState* gs;
  double* slab;
  RST_CHECK(b.get(sizeof(float) * 3 * n, (void**)&ds));
  RST_CHECK(b.get(sizeof(float) * 3 * m, (void**)&dd));
  RST_CHECK(b.get(sizeof(float) * 9 * n, (void**)&dcs));
  RST_CHECK(b.get(sizeof(float) * 9 * m, (void**)&dcd));
  RST_CHECK(b.get(sizeof(int32_t) * n, (void**)&di));
  RST_CHECK(b.get(sizeof(GicpState), (void**)&gs));
  RST_CHECK(b.get(sizeof(double) * kRS * (size_t)blocks_for(n), (void**)&slab));
  RST_CHECK(upload(st, ds, src, sizeof(float) * 3 * n));
  RST_CHECK(upload(st, dd, dst, sizeof(float) * 3 * m));
  RST_CHECK(upload(st, dcs, src_covs, sizeof(float) * 9 * n));
  RST_CHECK(upload(st, dcd, dst_covs, sizeof(float) * 9 * m));
  RST_CHECK(upload(st, di, dst_idx, sizeof(int32_t) * n));
  GicpState h;
  memset(&h, 0, sizeof(h));
  memcpy(h.est, seed, sizeof(h.est));
  RST_CHECK(upload(st, gs, &h, sizeof(h)));
  RST_CHECK(lm_solve(ctx, ds, n, dd, dcs, dcd, di, gs, slab, max_iter));
  RST_HIP(hipMemcpyAsync(&h, gs, sizeof(h), hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  memcpy(pose_out, h.est, sizeof(h.est));
  if (cost_out) *cost_out = h.F;
  if (iters_out) *iters_out = h.iters;
  for (int k = 0; k < 16; ++k)
    if (!std::isfinite(pose_out[k])) return RST_FALSE;
  return RST_OK;
}

int rst_gicp_align(rst_ctx* ctx, const float* src, int64_t n, const float* dst, int64_t m,
                   int outer_iters, int max_inner, float pose_out[16], double* cost_out) {
  if (!ctx || !src || !dst || !pose_out || n < 1 || m < 1 || outer_iters < 0 || max_inner < 1)
    return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  Bufs b;
  b.ctx = ctx;
  float *ds, *dd, *dcs, *dcd, *dtmp, *dd2;
  int32_t* di;
  GicpState* gs;
  double* slab;
  RST_CHECK(b.get(sizeof(float) * 3 * n, (void**)&ds));
  RST_CHECK(b.get(sizeof(float) * 3 * m, (void**)&dd));
  RST_CHECK(b.get(sizeof(float) * 9 * n, (void**)&dcs));
  RST_CHECK(b.get(sizeof(float) * 9 * m, (void**)&dcd));
  RST_CHECK(b.get(sizeof(float) * 3 * n + sizeof(float) * n, (void**)&dtmp));
  dd2 = dtmp + 3 * n;
  RST_CHECK(b.get(sizeof(int32_t) * n, (void**)&di));
  RST_CHECK(b.get(sizeof(GicpState) + sizeof(double) * kRS * (size_t)blocks_for(n), (void**)&gs));
  slab = (double*)(gs + 1);
  RST_CHECK(upload(st, ds, src, sizeof(float) * 3 * n));
  RST_CHECK(upload(st, dd, dst, sizeof(float) * 3 * m));
  // (:112-123) indices of both clouds, covariances (k = 32, use_gicp = false).
  // Small finite clouds (the downsampled frames) need no index: the
  // wave-per-point kernels scan them whole, in input order
  auto finite_all = [](const float* a, int64_t k) {
    for (int64_t i = 0; i < 3 * k; ++i)
      if (!std::isfinite(a[i])) return false;
    return true;
  };
  const bool flat = n <= kCovWaveMax && m <= kCovWaveMax && finite_all(src, n) &&
                    finite_all(dst, m);
  rst_target *ts = nullptr, *td = nullptr;
  BvhView vd = {};
  int s = RST_OK;
  if (flat) {
    float4 *s4 = nullptr, *d4 = nullptr;
    RST_CHECK(b.get(sizeof(float4) * n, (void**)&s4));
    RST_CHECK(b.get(sizeof(float4) * m, (void**)&d4));
    k_pack4<<<blocks_for(n), kBS, 0, st>>>(ds, n, s4);
    k_pack4<<<blocks_for(m), kBS, 0, st>>>(dd, m, d4);
    BvhView vs = {};
    vs.pts = s4;
    vs.m = (int32_t)n;
    vd.pts = d4;
    vd.m = (int32_t)m;
    k_covariances_wave<<<(unsigned)n, kWave, sizeof(uint64_t) * n, st>>>(vs, 0, 0, dcs);
    k_covariances_wave<<<(unsigned)m, kWave, sizeof(uint64_t) * m, st>>>(vd, 0, 0, dcd);
    if (hipGetLastError() != hipSuccess) s = RST_E_HIP;
  } else {
    s = target_build_device(ctx, ds, n, true, &ts);
    if (s >= 0) s = target_build_device(ctx, dd, m, true, &td);
    if (s >= 0) s = compute_covariances_device(ctx, ts, 0, dcs);
    if (s >= 0) s = compute_covariances_device(ctx, td, 0, dcd);
    if (s >= 0) vd = view_of(td);
  }
  // (:127-160) estimate = Identity; outer loop
  GicpState h;
  memset(&h, 0, sizeof(h));
  h.est[0] = h.est[5] = h.est[10] = h.est[15] = 1.f;
  if (s >= 0) s = upload(st, gs, &h, sizeof(h));
  for (int o = 0; s >= 0 && o < outer_iters; ++o) {
    k_gicp_xform<<<blocks_for(n), kBS, 0, st>>>(ds, n, gs, dtmp);
    // FindCorrespondences (:140-141): exact NN, from the last round's
    // neighbours after the first (the estimate moves little between rounds)
    if (m <= kCovWaveMax) {
      k_query_nn_wave<<<(unsigned)((n + kBS / kWave - 1) / (kBS / kWave)), kBS, 0, st>>>(
          vd, dtmp, n, di, dd2);
      s = hipGetLastError() == hipSuccess ? RST_OK : RST_E_HIP;
    } else {
      s = o == 0 ? query_nn_device(ctx, td, dtmp, n, di, dd2)
                 : query_nn_warm_device(ctx, td, dtmp, n, di, di, dd2);
    }
    if (s >= 0) s = lm_solve(ctx, ds, n, dd, dcs, dcd, di, gs, slab, max_inner);
  }
  if (s >= 0 && hipMemcpyAsync(&h, gs, sizeof(h), hipMemcpyDeviceToHost, st) != hipSuccess)
    s = RST_E_HIP;
  hipStreamSynchronize(st);
  if (ts) rst_target_free(ts);
  if (td) rst_target_free(td);
  if (s < 0) return s;
  memcpy(pose_out, h.est, sizeof(h.est));
  if (cost_out) *cost_out = outer_iters > 0 ? h.F : 0.0;
  for (int k = 0; k < 16; ++k)
    if (!std::isfinite(pose_out[k])) {  // (:145-150)
      if (cost_out) *cost_out = INFINITY;
      return RST_FALSE;
    }
  return RST_OK;
}

}  // extern "C"
