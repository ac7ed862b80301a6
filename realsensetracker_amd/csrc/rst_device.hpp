// rst_device.hpp -- device-side building blocks shared by the kernels.
//
// Arithmetic that must round exactly like the reference is written out
// operation by operation; the library is compiled with -ffp-contract=off so
// no multiply-add is fused behind our back (the reference is built for
// baseline x86-64: SSE2, no FMA).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include <type_traits>

#include "rst_bvh.hpp"

namespace rst {

// A pointer field of an argument struct read from device memory, typed as a
// global (address space 1) pointer: a pointer loaded from memory is generic,
// and every access through it a flat_load / flat_store -- which counts on
// lgkmcnt as well as vmcnt, so each LDS or scalar wait also waits for the
// memory loads in flight.  Only for fields that hold hipMalloc'd memory
// (null stays null).  The round trip through an integer keeps the compiler
// from folding the cast away; its address-space inference carries "global"
// into the inlined bodies (the batched kernels, icp.hip / seqsum.hip).
#ifndef RST_FLAT_ARGS
#define RST_FLAT_ARGS 0  // 1: the batched kernels' accesses flat again (measurement only)
#endif
template <class P>
__device__ __forceinline__ P as_glb(const P& field) {
  if (RST_FLAT_ARGS) return field;
  using T = typename std::remove_pointer<P>::type;
  typedef __attribute__((address_space(1))) T GT;
  GT* g = (GT*)(uintptr_t)field;
  return (P)g;
}

constexpr int kWave = 64;

// ---- pose application ----------------------------------------------------
// Transform<float,3,Isometry> * Vector3f: res = t; res += R*v, each coeff of
// the lazy 3x3 product an unrolled redux x0 + (x1 + x2)
// (align_icp.cpp:107, Eigen transform_right_product_impl).
__device__ __forceinline__ float mv_row(const float* R, int r, float v0,
                                        float v1, float v2) {
  const float a0 = R[0 * 3 + r] * v0;
  const float a1 = R[1 * 3 + r] * v1;
  const float a2 = R[2 * 3 + r] * v2;
  return a0 + (a1 + a2);
}

struct Pose3 {
  float r[9];
  float t[3];
};

__device__ __forceinline__ void xform(const Pose3& P, float sx, float sy,
                                      float sz, float& px, float& py,
                                      float& pz) {
  px = P.t[0] + mv_row(P.r, 0, sx, sy, sz);
  py = P.t[1] + mv_row(P.r, 1, sx, sy, sz);
  pz = P.t[2] + mv_row(P.r, 2, sx, sy, sz);
}

// ---- wave / block reductions ------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, kWave));
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// ---- transpose-reduce: NV sums over a wavefront in ~NV cross-lane moves ----
// A plain per-value butterfly costs 6 lane exchanges per value (6 NV
// ds_bpermute pairs for doubles).  Here every exchange step also halves the
// number of values a lane carries: at the step pairing lanes l and l ^ m,
// the lane without bit m keeps the lower half of its values and adds its
// partner's copy of that half, the other lane the upper half.  After
// log2(NV) such steps a lane carries one value -- the partial sum of value
// (lane >> (6 - log2 NV)) -- and the remaining steps reduce it plainly.
// Exchanges: v_permlane32_swap (lanes 32-63 of one register <-> lanes 0-31
// of another) and v_permlane16_swap (the same between adjacent 16-lane
// rows) pair whole registers, so each half-step is one swap per dword;
// inside a row DPP row_mirror (l <-> 15 - l), row_half_mirror (l <-> 7 - l)
// and quad_perm do the rest -- no LDS traffic.  Bitwise deterministic.
__device__ __forceinline__ void swap_halves32(double& a, double& b) {
  uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
  const auto rx = __builtin_amdgcn_permlane32_swap(ua.x, ub.x, false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(ua.y, ub.y, false, false);
  a = __builtin_bit_cast(double, make_uint2(rx[0], ry[0]));
  b = __builtin_bit_cast(double, make_uint2(rx[1], ry[1]));
}
__device__ __forceinline__ void swap_rows16(double& a, double& b) {
  uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
  const auto rx = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
  a = __builtin_bit_cast(double, make_uint2(rx[0], ry[0]));
  b = __builtin_bit_cast(double, make_uint2(rx[1], ry[1]));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const uint2 u = __builtin_bit_cast(uint2, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u.x, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)u.y, CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, make_uint2((unsigned)lo, (unsigned)hi));
}
constexpr int kDppRowMirror = 0x140, kDppRowHalfMirror = 0x141;
constexpr int kDppXor2 = 0x4E, kDppXor1 = 0xB1;  // quad_perm [2,3,0,1] / [1,0,3,2]

// One step of the transpose-reduce: `cnt` values in v[0..cnt) -> cnt / 2
// (or, at cnt == 1, a plain pairwise sum).  STEP 0..5 pairs lanes across
// bit 5 .. bit 0 of the lane id.
template <int STEP, int N>
__device__ __forceinline__ void transpose_step(double (&v)[N], int cnt, int lane) {
  const int h = cnt > 1 ? cnt / 2 : 1;
  if (cnt == 1) {
    double a = v[0];
    if constexpr (STEP == 0) {
      double b = a;
      swap_halves32(a, b);
      v[0] = a + b;
    } else if constexpr (STEP == 1) {
      double b = a;
      swap_rows16(a, b);
      v[0] = a + b;
    } else if constexpr (STEP == 2) {
      v[0] = a + dpp_f64<kDppRowMirror>(a);
    } else if constexpr (STEP == 3) {
      v[0] = a + dpp_f64<kDppRowHalfMirror>(a);
    } else if constexpr (STEP == 4) {
      v[0] = a + dpp_f64<kDppXor2>(a);
    } else {
      v[0] = a + dpp_f64<kDppXor1>(a);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < N / 2; ++j) {
    if (j >= h) break;
    if constexpr (STEP == 0) {
      swap_halves32(v[j], v[j + h]);
      v[j] = v[j] + v[j + h];
    } else if constexpr (STEP == 1) {
      swap_rows16(v[j], v[j + h]);
      v[j] = v[j] + v[j + h];
    } else {
      const bool up = (lane >> (5 - STEP)) & 1;  // keeps the upper half
      const double send = up ? v[j] : v[j + h];
      double recv;
      if constexpr (STEP == 2)
        recv = dpp_f64<kDppRowMirror>(send);
      else if constexpr (STEP == 3)
        recv = dpp_f64<kDppRowHalfMirror>(send);
      else if constexpr (STEP == 4)
        recv = dpp_f64<kDppXor2>(send);
      else
        recv = dpp_f64<kDppXor1>(send);
      v[j] = (up ? v[j + h] : v[j]) + recv;
    }
  }
}

constexpr int pow2_ceil(int x) { return x <= 1 ? 1 : 2 * pow2_ceil((x + 1) / 2); }
constexpr int log2_exact(int x) { return x <= 1 ? 0 : 1 + log2_exact(x / 2); }

// Wave sums of NV doubles: returns the total of value (lane >> (6 - k)),
// k = log2(pow2_ceil(NV)), held by every lane of that group (the caller
// writes it from lanes with (lane & ((1 << (6 - k)) - 1)) == 0).
template <int NV>
__device__ __forceinline__ double wave_sum_transpose(const double (&v)[NV], int lane) {
  constexpr int P = pow2_ceil(NV);
  static_assert(P <= kWave, "at most 64 values");
  double w[P];
#pragma unroll
  for (int k = 0; k < P; ++k) w[k] = k < NV ? v[k] : 0.0;
  int cnt = P;
  transpose_step<0>(w, cnt, lane);
  cnt = cnt > 1 ? cnt / 2 : 1;
  transpose_step<1>(w, cnt, lane);
  cnt = cnt > 1 ? cnt / 2 : 1;
  transpose_step<2>(w, cnt, lane);
  cnt = cnt > 1 ? cnt / 2 : 1;
  transpose_step<3>(w, cnt, lane);
  cnt = cnt > 1 ? cnt / 2 : 1;
  transpose_step<4>(w, cnt, lane);
  cnt = cnt > 1 ? cnt / 2 : 1;
  transpose_step<5>(w, cnt, lane);
  return w[0];
}

// Reduce NV doubles per thread over a block of BS threads; lane results land
// in out[] on thread 0..NV-1 (out must be __shared__ double[BS/64][NV]).
template <int NV, int BS>
__device__ __forceinline__ void block_sum_to_slab(double (&v)[NV],
                                                  double* lds,
                                                  double* slab_row) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  constexpr int K = log2_exact(pow2_ceil(NV));
  const double t = wave_sum_transpose<NV>(v, lane);
  const int idx = lane >> (6 - K);
  if ((lane & ((1 << (6 - K)) - 1)) == 0 && idx < NV) lds[wid * NV + idx] = t;
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < BS / kWave; ++w) s += lds[w * NV + threadIdx.x];
    slab_row[threadIdx.x] = s;
  }
}

// block_sum_to_slab added onto the row's current values (a later kernel's
// share of the same tile: fixed order, reproducible)
template <int NV, int BS>
__device__ __forceinline__ void block_sum_add_to_slab(double (&v)[NV], double* lds,
                                                      double* slab_row) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  constexpr int K = log2_exact(pow2_ceil(NV));
  const double old = threadIdx.x < NV ? slab_row[threadIdx.x] : 0.0;  // in flight meanwhile
  const double t = wave_sum_transpose<NV>(v, lane);
  const int idx = lane >> (6 - K);
  if ((lane & ((1 << (6 - K)) - 1)) == 0 && idx < NV) lds[wid * NV + idx] = t;
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < BS / kWave; ++w) s += lds[w * NV + threadIdx.x];
    slab_row[threadIdx.x] = old + s;
  }
}

// block_sum_to_slab, then rows blk, blk + step, ... (< rows) of another slab
// (row stride `stride`) added in increasing order: a grid of G blocks folds
// an earlier kernel's rows into its own G, fixed order (reproducible).
template <int NV, int BS>
__device__ __forceinline__ void block_sum_to_slab_fold(double (&v)[NV], double* lds,
                                                       double* slab_row,
                                                       const double* __restrict__ other,
                                                       int rows, int stride, int blk, int step) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  double ex = 0.0;  // loads issued before the wave sums (latency overlap)
  if (threadIdx.x < NV)
    for (int r = blk; r < rows; r += step) ex += other[(int64_t)r * stride + threadIdx.x];
  constexpr int K = log2_exact(pow2_ceil(NV));
  const double t = wave_sum_transpose<NV>(v, lane);
  const int idx = lane >> (6 - K);
  if ((lane & ((1 << (6 - K)) - 1)) == 0 && idx < NV) lds[wid * NV + idx] = t;
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < BS / kWave; ++w) s += lds[w * NV + threadIdx.x];
    slab_row[threadIdx.x] = s + ex;
  }
}

// ---- 3x3 linear algebra (single thread) -------------------------------------
#define RST_M3(m, r, c) (m)[(c) * 3 + (r)]

// One-sided Jacobi SVD of a 3x3 double matrix (column-major):
// a = U diag(s) V^T.  Columns of a are orthogonalised by plane rotations
// accumulated in V; U = normalised columns.  Rank-2 input: the missing U
// column is completed as the cross product of the other two.
__device__ inline void svd3_jacobi(const double* a_in, double* U, double* S,
                                   double* V) {
  double A[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    A[i] = a_in[i];
    V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  }
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0;
#pragma unroll
    for (int pr = 0; pr < 3; ++pr) {
      const int p = pr == 2 ? 1 : 0;
      const int q = pr == 0 ? 1 : 2;
      double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        alpha += RST_M3(A, r, p) * RST_M3(A, r, p);
        beta += RST_M3(A, r, q) * RST_M3(A, r, q);
        gamma += RST_M3(A, r, p) * RST_M3(A, r, q);
      }
      const double denom = sqrt(alpha * beta);
      if (denom == 0.0 || fabs(gamma) <= 1e-15 * denom) continue;
      off = fmax(off, fabs(gamma) / denom);
      const double zeta = (beta - alpha) / (2.0 * gamma);
      const double tt = (zeta >= 0 ? 1.0 : -1.0) /
                        (fabs(zeta) + sqrt(1.0 + zeta * zeta));
      const double c = 1.0 / sqrt(1.0 + tt * tt);
      const double s = c * tt;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double ap = RST_M3(A, r, p), aq = RST_M3(A, r, q);
        RST_M3(A, r, p) = c * ap - s * aq;
        RST_M3(A, r, q) = s * ap + c * aq;
        const double vp = RST_M3(V, r, p), vq = RST_M3(V, r, q);
        RST_M3(V, r, p) = c * vp - s * vq;
        RST_M3(V, r, q) = s * vp + c * vq;
      }
    }
    if (off <= 1e-15) break;
  }
  double smax = 0.0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double n2 = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) n2 += RST_M3(A, r, c) * RST_M3(A, r, c);
    S[c] = sqrt(n2);
    smax = fmax(smax, S[c]);
  }
  const double tiny = smax * 1e-13;
  int nz = 0, zc = -1;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (S[c] > tiny && S[c] > 0.0) {
#pragma unroll
      for (int r = 0; r < 3; ++r) RST_M3(U, r, c) = RST_M3(A, r, c) / S[c];
      ++nz;
    } else {
#pragma unroll
      for (int r = 0; r < 3; ++r) RST_M3(U, r, c) = 0.0;
      zc = c;
    }
  }
  if (nz <= 1) {
    // rank <= 1: degenerate; U = V gives R = U V^T = I (what an all-zero
    // covariance yields in the reference, whose Jacobi SVD then does nothing)
#pragma unroll
    for (int i = 0; i < 9; ++i) U[i] = V[i];
  } else if (nz == 2) {
    // u_z = u_c0 x u_c1, in the cyclic orientation of (c0, c1, zc), with
    // c0 = first and c1 = second non-zero column (selects, not indices:
    // every array index stays static, so nothing lands in scratch memory)
    double a[3], b[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      a[r] = zc == 0 ? RST_M3(U, r, 1) : RST_M3(U, r, 0);
      b[r] = zc == 2 ? RST_M3(U, r, 1) : RST_M3(U, r, 2);
    }
    double x[3];
    x[0] = a[1] * b[2] - a[2] * b[1];
    x[1] = a[2] * b[0] - a[0] * b[2];
    x[2] = a[0] * b[1] - a[1] * b[0];
    const double sg = (zc == 1) ? -1.0 : 1.0;  // (0,2,1) is an odd order
    // keep det(U) == det(V) so U V^T is a proper rotation
    double dv = RST_M3(V, 0, 0) * (RST_M3(V, 1, 1) * RST_M3(V, 2, 2) - RST_M3(V, 1, 2) * RST_M3(V, 2, 1)) -
                RST_M3(V, 0, 1) * (RST_M3(V, 1, 0) * RST_M3(V, 2, 2) - RST_M3(V, 1, 2) * RST_M3(V, 2, 0)) +
                RST_M3(V, 0, 2) * (RST_M3(V, 1, 0) * RST_M3(V, 2, 1) - RST_M3(V, 1, 1) * RST_M3(V, 2, 0));
    const double sd = dv < 0 ? -1.0 : 1.0;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (c == zc) RST_M3(U, r, c) = sg * sd * x[r];
  }
}

// Orthogonal polar factor Q of a nonsingular 3x3 a (column-major), i.e.
// U V^T of its SVD, by scaled Newton iteration X <- (g X + X^-T / g) / 2
// (Higham; g = sqrt(|X^-1|_F / |X|_F) while far from convergence, then 1
// for the quadratic tail).  For nonsingular a the polar factor is unique, so
// this is the same rotation JacobiSVD's U V^T gives (align_icp.cpp:139-141)
// at ~1e-16 relative; a few dozen fp64 flops per step instead of Jacobi
// sweeps.  Returns false (the caller falls back to svd3_jacobi) when a is
// numerically singular or the iteration does not settle.
#ifndef RST_POLAR_MIN_IT
#define RST_POLAR_MIN_IT 1  // r01h A/B: 6 -> 1 cut the solve 5.3 -> 4.6 us
#endif
constexpr int kPolarScaled = 6;                 // scaled Newton steps (then g = 1)
constexpr int kPolarMinIt = RST_POLAR_MIN_IT;   // earliest converged exit
__device__ __forceinline__ bool polar3(const double* a, double* Q) {
  double X[9];
  double nx = 0.0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    X[i] = a[i];
    nx += a[i] * a[i];
  }
  nx = sqrt(nx);
  if (!(nx > 0.0) || !(nx < 1e300)) return false;
  for (int it = 0; it < 40; ++it) {
    // cofactor matrix C (column-major): X^-T = C / det
    double C[9];
    RST_M3(C, 0, 0) = RST_M3(X, 1, 1) * RST_M3(X, 2, 2) - RST_M3(X, 1, 2) * RST_M3(X, 2, 1);
    RST_M3(C, 0, 1) = RST_M3(X, 1, 2) * RST_M3(X, 2, 0) - RST_M3(X, 1, 0) * RST_M3(X, 2, 2);
    RST_M3(C, 0, 2) = RST_M3(X, 1, 0) * RST_M3(X, 2, 1) - RST_M3(X, 1, 1) * RST_M3(X, 2, 0);
    RST_M3(C, 1, 0) = RST_M3(X, 0, 2) * RST_M3(X, 2, 1) - RST_M3(X, 0, 1) * RST_M3(X, 2, 2);
    RST_M3(C, 1, 1) = RST_M3(X, 0, 0) * RST_M3(X, 2, 2) - RST_M3(X, 0, 2) * RST_M3(X, 2, 0);
    RST_M3(C, 1, 2) = RST_M3(X, 0, 1) * RST_M3(X, 2, 0) - RST_M3(X, 0, 0) * RST_M3(X, 2, 1);
    RST_M3(C, 2, 0) = RST_M3(X, 0, 1) * RST_M3(X, 1, 2) - RST_M3(X, 0, 2) * RST_M3(X, 1, 1);
    RST_M3(C, 2, 1) = RST_M3(X, 0, 2) * RST_M3(X, 1, 0) - RST_M3(X, 0, 0) * RST_M3(X, 1, 2);
    RST_M3(C, 2, 2) = RST_M3(X, 0, 0) * RST_M3(X, 1, 1) - RST_M3(X, 0, 1) * RST_M3(X, 1, 0);
    const double det = RST_M3(X, 0, 0) * RST_M3(C, 0, 0) + RST_M3(X, 0, 1) * RST_M3(C, 0, 1) +
                       RST_M3(X, 0, 2) * RST_M3(C, 0, 2);
    double n2 = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) n2 += X[i] * X[i];
    // (norms and the scale in fp32: they only steer the convergence -- any
    // g > 0 keeps the polar factor -- and the singularity test is a bound)
    const float nXf = n2 < 1e30 ? sqrtf((float)n2) : (float)sqrt(n2);
    const double nX = (double)nXf;
    // numerically singular (condition ~ nX^3 / |det| beyond ~1e12)
    if (!(fabs(det) > 1e-12 * nX * nX * nX)) return false;
    const double id = 1.0 / det;
    double ni2 = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      C[i] *= id;
      ni2 += C[i] * C[i];
    }
    const double g =
        it < kPolarScaled ? (double)sqrtf(sqrtf((float)fmin(ni2, 1e30)) / nXf) : 1.0;
    const double ig = 1.0 / g;
    double diff = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const double xn = 0.5 * (g * X[i] + C[i] * ig);
      diff += (xn - X[i]) * (xn - X[i]);
      X[i] = xn;
    }
    // quadratic convergence: a step that moved X by <= ~1e-9 leaves it
    // within ~1e-18 of the polar factor, below fp64 resolution
    if (it >= kPolarMinIt && diff <= 1e-18) {
#pragma unroll
      for (int i = 0; i < 9; ++i) Q[i] = X[i];
      return true;
    }
  }
  return false;
}

// Matrix3f::determinant (Eigen bruteforce_det3_helper order).
__device__ __forceinline__ float det3f(const float* m) {
  const float d0 = RST_M3(m, 0, 0) * (RST_M3(m, 1, 1) * RST_M3(m, 2, 2) - RST_M3(m, 1, 2) * RST_M3(m, 2, 1));
  const float d1 = RST_M3(m, 0, 1) * (RST_M3(m, 1, 0) * RST_M3(m, 2, 2) - RST_M3(m, 1, 2) * RST_M3(m, 2, 0));
  const float d2 = RST_M3(m, 0, 2) * (RST_M3(m, 1, 0) * RST_M3(m, 2, 1) - RST_M3(m, 1, 1) * RST_M3(m, 2, 0));
  return (d0 - d1) + d2;
}

// Quaternionf(R) then toRotationMatrix() (align_icp.cpp:151; Eigen
// quaternionbase_assign_impl<3x3> / toRotationMatrix op order).
__device__ __forceinline__ void quat_roundtrip(const float* R, float* Rq) {
  float q[4];  // x y z w
  const float tr = (RST_M3(R, 0, 0) + RST_M3(R, 1, 1)) + RST_M3(R, 2, 2);
  if (tr > 0.0f) {
    float t = sqrtf(tr + 1.0f);
    q[3] = 0.5f * t;
    t = 0.5f / t;
    q[0] = (RST_M3(R, 2, 1) - RST_M3(R, 1, 2)) * t;
    q[1] = (RST_M3(R, 0, 2) - RST_M3(R, 2, 0)) * t;
    q[2] = (RST_M3(R, 1, 0) - RST_M3(R, 0, 1)) * t;
  } else {
    // i = argmax diagonal, j = i+1, k = i+2 (mod 3), spelled out per i so
    // every index is static (no scratch memory on the GPU)
    int i = 0;
    if (RST_M3(R, 1, 1) > RST_M3(R, 0, 0)) i = 1;
    if (RST_M3(R, 2, 2) > (i == 0 ? RST_M3(R, 0, 0) : RST_M3(R, 1, 1))) i = 2;
    if (i == 0) {
      float t = sqrtf(RST_M3(R, 0, 0) - RST_M3(R, 1, 1) - RST_M3(R, 2, 2) + 1.0f);
      q[0] = 0.5f * t;
      t = 0.5f / t;
      q[3] = (RST_M3(R, 2, 1) - RST_M3(R, 1, 2)) * t;
      q[1] = (RST_M3(R, 1, 0) + RST_M3(R, 0, 1)) * t;
      q[2] = (RST_M3(R, 2, 0) + RST_M3(R, 0, 2)) * t;
    } else if (i == 1) {
      float t = sqrtf(RST_M3(R, 1, 1) - RST_M3(R, 2, 2) - RST_M3(R, 0, 0) + 1.0f);
      q[1] = 0.5f * t;
      t = 0.5f / t;
      q[3] = (RST_M3(R, 0, 2) - RST_M3(R, 2, 0)) * t;
      q[2] = (RST_M3(R, 2, 1) + RST_M3(R, 1, 2)) * t;
      q[0] = (RST_M3(R, 0, 1) + RST_M3(R, 1, 0)) * t;
    } else {
      float t = sqrtf(RST_M3(R, 2, 2) - RST_M3(R, 0, 0) - RST_M3(R, 1, 1) + 1.0f);
      q[2] = 0.5f * t;
      t = 0.5f / t;
      q[3] = (RST_M3(R, 1, 0) - RST_M3(R, 0, 1)) * t;
      q[0] = (RST_M3(R, 0, 2) + RST_M3(R, 2, 0)) * t;
      q[1] = (RST_M3(R, 1, 2) + RST_M3(R, 2, 1)) * t;
    }
  }
  const float x = q[0], y = q[1], z = q[2], w = q[3];
  const float tx = 2.0f * x, ty = 2.0f * y, tz = 2.0f * z;
  const float twx = tx * w, twy = ty * w, twz = tz * w;
  const float txx = tx * x, txy = ty * x, txz = tz * x;
  const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
  RST_M3(Rq, 0, 0) = 1.0f - (tyy + tzz);
  RST_M3(Rq, 0, 1) = txy - twz;
  RST_M3(Rq, 0, 2) = txz + twy;
  RST_M3(Rq, 1, 0) = txy + twz;
  RST_M3(Rq, 1, 1) = 1.0f - (txx + tzz);
  RST_M3(Rq, 1, 2) = tyz - twx;
  RST_M3(Rq, 2, 0) = txz - twy;
  RST_M3(Rq, 2, 1) = tyz + twx;
  RST_M3(Rq, 2, 2) = 1.0f - (txx + tyy);
}

}  // namespace rst
