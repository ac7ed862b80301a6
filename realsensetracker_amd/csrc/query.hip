// query.hip -- exact NN / kNN queries against a target index and kNN-PCA
// normals.
//
//   query_nn_device  : KDTree3f::query(p, 1, &j, &d2)  (kdtree.hpp:51-57)
//   query_knn_device : KDTree3f index->knnSearch(p, k, ...) (fpfh/normals)
//   compute_normals  : ComputeNormals + OrientNormals
//                      (point_cloud_utils.cpp:176-216)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "rst_device.hpp"
#include "rst_wave_nn.hpp"
#include "rst_internal.hpp"

namespace rst {
namespace {

constexpr int kBS = 256;

// One query per lane, top-down from the root (no warm candidate).
__global__ __launch_bounds__(kBS) void k_query_nn(BvhView bv, const float* __restrict__ q,
                                                  int64_t nq, int32_t* __restrict__ idx,
                                                  float* __restrict__ d2) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= nq) return;
  Best1 r;
  r.init();
  search(bv, -1, q[3 * i], q[3 * i + 1], q[3 * i + 2], r);
  idx[i] = r.id;
  d2[i] = r.d;
}

// Coherent queries with warm candidates (original target indices, <0 or
// out of range = none): the wave-cooperative search the ICP loop uses.
__global__ __launch_bounds__(kBS) void k_query_nn_warm(BvhView bv, const int32_t* __restrict__ inv,
                                                       const float* __restrict__ q, int64_t nq,
                                                       const int32_t* __restrict__ warm,
                                                       int32_t* __restrict__ idx,
                                                       float* __restrict__ d2,
                                                       int* __restrict__ stats) {
  __shared__ WnnScratch wsc[kBS / kWave];
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  const bool act = i < nq;
  float qx = 0.f, qy = 0.f, qz = 0.f;
  Best1 r;
  r.init();
  if (act) {
    qx = q[3 * i];
    qy = q[3 * i + 1];
    qz = q[3 * i + 2];
    const int w = warm ? warm[i] : -1;
    if (w >= 0 && w < bv.m) {
      const int pos = inv[w];
      const float4 p = bv.pts[pos];
      r.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), pos);
    }
  }
  nn_wave_region(bv, act, qx, qy, qz, r, wsc[threadIdx.x / kWave],
                 stats ? stats + 8 * (int64_t)(i / kWave) : nullptr);
  if (act) {
    idx[i] = r.id;
    d2[i] = r.d;
  }
}

// The ICP fallback's per-query searches (icp.hip k_icp_fb), one wavefront
// per query, for testing: mode 0 = the full walk from the warm leaf; 2 / 3 =
// the level-2 / level-3 adjacency first (then the walk when not covered);
// 23 = level 2, then 3, then the walk (what the ICP loop does).  path[i] =
// the strategy that answered (2, 3 or 0).
__global__ __launch_bounds__(kBS) void k_query_nn_fallback(BvhView bv, AdjView av,
                                                           const int32_t* __restrict__ inv,
                                                           const float* __restrict__ q,
                                                           int64_t nq,
                                                           const int32_t* __restrict__ warm,
                                                           int mode, int32_t* __restrict__ idx,
                                                           float* __restrict__ d2,
                                                           int32_t* __restrict__ path) {
  __shared__ WnnScratch wsc[kBS / kWave];
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int64_t i = blockIdx.x * (int64_t)(kBS / kWave) + wid;
  if (i >= nq) return;  // wave-uniform
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
  int start = -1;
  const int w = warm ? warm[i] : -1;
  const bool seeded = w >= 0 && w < bv.m && finite3(qx, qy, qz);
  if (seeded) start = inv[w];
  if (mode >= 1000) {  // the two nearest, seeded like the ICP loop (warm + its sorted neighbour)
    Best2 r2;
    r2.init();
    if (seeded) {
      const float4 p = bv.pts[start];
      r2.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), start);
      if (bv.m > 1) {
        const int nb = start + 1 < bv.m ? start + 1 : start - 1;
        const float4 p2 = bv.pts[nb];
        r2.offer(d2_ref(qx, qy, qz, p2.x, p2.y, p2.z), f2i(p2.w), nb);
      }
    }
    if (!nn_wave_adj(bv, av, kAdj2Shift, start, qx, qy, qz, r2, wsc[wid]) &&
        !nn_wave_adj(bv, av, kAdj3Shift, start, qx, qy, qz, r2, wsc[wid]))
      nn_wave_one(bv, start, qx, qy, qz, r2, wsc[wid]);
    if (lane == 0) {
      const Best1 r = r2.first();
      idx[i] = r.id;
      d2[i] = r.d;
      path[i] = __float_as_int(r2.d[1]);  // the second-nearest d2 (bits)
    }
    return;
  }
  Best1 r;
  r.init();
  if (seeded) {
    const float4 p = bv.pts[start];
    r.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), start);
  }
  int how = 0;
  if ((mode == 2 || mode == 23) && nn_wave_adj(bv, av, kAdj2Shift, start, qx, qy, qz, r, wsc[wid]))
    how = 2;
  else if ((mode == 3 || mode == 23) &&
           nn_wave_adj(bv, av, kAdj3Shift, start, qx, qy, qz, r, wsc[wid]))
    how = 3;
  else
    nn_wave_one(bv, start, qx, qy, qz, r, wsc[wid], mode >= 100 ? mode - 100 : 0);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    idx[i] = r.pos >= 0 ? r.id : 0;
    d2[i] = r.d;
    // strategy in the low 4 bits, the wave's shader cycles / 16 above
    uint64_t c16 = (t1 - t0) >> 4;
    if (c16 > (uint64_t)((1u << 27) - 1)) c16 = (1u << 27) - 1;
    path[i] = how | ((int)c16 << 4);
  }
}

template <int K>
__global__ __launch_bounds__(kBS) void k_query_knn(BvhView bv, const float* __restrict__ q,
                                                   int64_t nq, int k,
                                                   int32_t* __restrict__ idx,
                                                   float* __restrict__ d2) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= nq) return;
  BestK<K> L;
  L.init();
  search(bv, -1, q[3 * i], q[3 * i + 1], q[3 * i + 2], L);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (j < k) {
      const bool filled = L.pos[j] >= 0;
      idx[i * k + j] = filled ? L.id[j] : 0;
      d2[i * k + j] = filled ? L.d[j] : FLT_MAX;
    }
  }
}

// Smallest-eigenvalue eigenvector of a symmetric 3x3 (double): eigenvalues
// from the trigonometric closed form, eigenvector as the best-conditioned
// cross product of rows of (A - lambda I).
__device__ inline void sym3_min_vec(const double a[6], double v[3]) {
  // a = {xx, xy, xz, yy, yz, zz}
  const double xx = a[0], xy = a[1], xz = a[2], yy = a[3], yz = a[4], zz = a[5];
  const double p1 = xy * xy + xz * xz + yz * yz;
  const double q = (xx + yy + zz) / 3.0;
  const double p2 = (xx - q) * (xx - q) + (yy - q) * (yy - q) + (zz - q) * (zz - q) + 2.0 * p1;
  const double p = sqrt(p2 / 6.0);
  double lmin;
  if (p < 1e-300) {
    v[0] = 0.0; v[1] = 0.0; v[2] = 1.0;
    return;
  }
  {
    const double bxx = (xx - q) / p, byy = (yy - q) / p, bzz = (zz - q) / p;
    const double bxy = xy / p, bxz = xz / p, byz = yz / p;
    const double detb = bxx * (byy * bzz - byz * byz) - bxy * (bxy * bzz - byz * bxz) +
                        bxz * (bxy * byz - byy * bxz);
    double r = detb / 2.0;
    r = fmin(1.0, fmax(-1.0, r));
    const double phi = acos(r) / 3.0;
    lmin = q + 2.0 * p * cos(phi + 2.0 * M_PI / 3.0);
  }
  const double r0[3] = {xx - lmin, xy, xz};
  const double r1[3] = {xy, yy - lmin, yz};
  const double r2[3] = {xz, yz, zz - lmin};
  double c[3][3];
  c[0][0] = r0[1] * r1[2] - r0[2] * r1[1]; c[0][1] = r0[2] * r1[0] - r0[0] * r1[2]; c[0][2] = r0[0] * r1[1] - r0[1] * r1[0];
  c[1][0] = r0[1] * r2[2] - r0[2] * r2[1]; c[1][1] = r0[2] * r2[0] - r0[0] * r2[2]; c[1][2] = r0[0] * r2[1] - r0[1] * r2[0];
  c[2][0] = r1[1] * r2[2] - r1[2] * r2[1]; c[2][1] = r1[2] * r2[0] - r1[0] * r2[2]; c[2][2] = r1[0] * r2[1] - r1[1] * r2[0];
  int bi = 0;
  double bn = -1.0;
  for (int i = 0; i < 3; ++i) {
    const double n2 = c[i][0] * c[i][0] + c[i][1] * c[i][1] + c[i][2] * c[i][2];
    if (n2 > bn) {
      bn = n2;
      bi = i;
    }
  }
  if (bn < 1e-300) {
    v[0] = 0.0; v[1] = 0.0; v[2] = 1.0;
    return;
  }
  const double inv = 1.0 / sqrt(bn);
  v[0] = c[bi][0] * inv;
  v[1] = c[bi][1] * inv;
  v[2] = c[bi][2] * inv;
}

// The normal of point p from its K nearest (L, sorted by (d2, index)):
// centroid in result order, fp32 (point_cloud_utils.cpp:186-191), fp32
// outer-product covariance (:193-198), smallest-eigenvalue eigenvector,
// oriented as OrientNormals (:206-216): flip if (p - viewpoint).n > 0.
template <int K>
__device__ __forceinline__ float4 knn_normal(const BvhView& bv, const BestK<K>& L, const float4& p, float vx,
                                             float vy, float vz) {
  float cx = 0.f, cy = 0.f, cz = 0.f;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const float4 s = L.pos[j] >= 0 ? bv.pts[L.pos[j]] : make_float4(0.f, 0.f, 0.f, 0.f);
    cx += s.x;
    cy += s.y;
    cz += s.z;
  }
  const float kf = (float)K;
  cx = cx / kf;
  cy = cy / kf;
  cz = cz / kf;
  float c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const float4 s = L.pos[j] >= 0 ? bv.pts[L.pos[j]] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float dx = s.x - cx, dy = s.y - cy, dz = s.z - cz;
    c00 += dx * dx; c01 += dx * dy; c02 += dx * dz;
    c11 += dy * dy; c12 += dy * dz; c22 += dz * dz;
  }
  const double a[6] = {c00, c01, c02, c11, c12, c22};
  double v[3];
  sym3_min_vec(a, v);
  float nx = (float)v[0], ny = (float)v[1], nz = (float)v[2];
  const float rx = p.x - vx, ry = p.y - vy, rz = p.z - vz;
  const float dot = rx * nx + (ry * ny + rz * nz);
  if (dot > 0) {
    nx = -nx;
    ny = -ny;
    nz = -nz;
  }
  return make_float4(nx, ny, nz, 0.0f);
}

template <int K>
__global__ __launch_bounds__(kBS) void k_normals(BvhView bv, int64_t m, float vx, float vy,
                                                 float vz, float4* __restrict__ nrm) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= m) return;
  const float4 p = bv.pts[i];
  // the query is target point i itself: bottom-up from its own leaf
  BestK<K> L;
  L.init();
  search(bv, (int)i, p.x, p.y, p.z, L);
  nrm[i] = knn_normal<K>(bv, L, p, vx, vy, vz);
}

// ComputeNormals' exact kNN through a frame target's pixel grid (the
// reference's kd-tree search, kdtree.hpp:51-57, k = 16 at its call sites):
// every point of a frame lies on the ray of its pixel, so the K nearest of
// point p are found in a pixel window -- seeded by the 7 x 7 pixels around
// p's own (their K-th nearest bounds the K-th distance), then the window of
// that ball (pix_window: every target point within the radius projects
// inside it) scanned for the rest.  A 16 x 16 block of pixels stages its
// tile and an 8-pixel halo in LDS (one 16-byte load per pixel), so every
// window up to 8 pixels is scanned from LDS.  Candidates are ranked by (d2,
// original index) as the BVH search ranks them, so the K nearest -- and the
// normal -- are the same bits; a ball whose window is wider (depth edges,
// too few seeds) takes the BVH search.  r09: the BVH search per lane, 1.2 ms
// a 640x480 frame; r10: the windows per lane from global memory, 0.87 ms.
constexpr int kKnnT = 16;              // tile side (pixels)
constexpr int kKnnHalo = 8;            // staged halo = the widest window scanned
constexpr int kKnnTW = kKnnT + 2 * kKnnHalo;
constexpr int kKnnSeedR = 3;           // the seed: (2 r + 1)^2 pixels (7 x 7: beside a depth edge
                                       // ~half of them lie on the point's own surface, enough for 16)
template <int K>
__global__ __launch_bounds__(kKnnT* kKnnT) void k_normals_grid(BvhView bv, PixView pv, float vx, float vy,
                                                                float vz, float4* __restrict__ nrm,
                                                                int32_t* __restrict__ fbq) {
  __shared__ float4 tile[kKnnTW * kKnnTW];
  const int u0 = blockIdx.x * kKnnT - kKnnHalo, v0 = blockIdx.y * kKnnT - kKnnHalo;
  for (int k = threadIdx.x; k < kKnnTW * kKnnTW; k += kKnnT * kKnnT) {
    const int uu = u0 + k % kKnnTW, vv = v0 + k / kKnnTW;
    tile[k] = (uu >= 0 && vv >= 0 && uu < pv.w && vv < pv.h) ? pv.pts[(int64_t)vv * pv.w + uu]
                                                             : make_float4(NAN, NAN, NAN, 0.f);
  }
  __syncthreads();
  const int lu = threadIdx.x % kKnnT, lv = threadIdx.x / kKnnT;
  const int u = blockIdx.x * kKnnT + lu, v = blockIdx.y * kKnnT + lv;
  if (u >= pv.w || v >= pv.h) return;
  const int pos = pv.map[(int64_t)v * pv.w + u];
  if (pos < 0) return;
  const int tu = lu + kKnnHalo, tv = lv + kKnnHalo;  // the pixel in the tile
  const float4 p = tile[tv * kKnnTW + tu];
  BestK<K> L;
  L.init();
  bool done = false;
#pragma unroll
  for (int k = 0; k < (2 * kKnnSeedR + 1) * (2 * kKnnSeedR + 1); ++k) {
    const float4 q = tile[(tv + k / (2 * kKnnSeedR + 1) - kKnnSeedR) * kKnnTW + (tu + k % (2 * kKnnSeedR + 1) - kKnnSeedR)];
    const float d = d2_ref(p.x, p.y, p.z, q.x, q.y, q.z);  // (NaN: no point)
    if (d <= L.bound()) L.offer(d, f2i(q.w), kPosPending);
  }
  int a0, a1, b0, b1;
  float rc;
  if (pix_window(pv, p.x, p.y, p.z, L.bound(), (float)kKnnHalo, a0, a1, b0, b1, rc) && a0 >= u0 &&
      a1 < u0 + kKnnTW && b0 >= v0 && b1 < v0 + kKnnTW) {
    for (int b = b0; b <= b1; ++b) {
      const float4* row = tile + (b - v0) * kKnnTW - u0;
      const bool inrow = b >= v - kKnnSeedR && b <= v + kKnnSeedR;
      for (int a = a0; a <= a1; a += 4) {
        float4 t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int aa = a + j;
          const bool seen = inrow && aa >= u - kKnnSeedR && aa <= u + kKnnSeedR;  // (offered above)
          t[j] = aa <= a1 && !seen ? row[aa] : make_float4(NAN, NAN, NAN, 0.f);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = d2_ref(p.x, p.y, p.z, t[j].x, t[j].y, t[j].z);
          if (d <= L.bound()) L.offer(d, f2i(t[j].w), kPosPending);
        }
      }
    }
    // every one of the K within the covered radius (always, the seeds being
    // inside it; checked anyway)
    done = L.pos[K - 1] >= 0 && margin_sqrt(L.bound()) * 1.00001f + 1e-30f < rc;
  }
  if (done) {
#pragma unroll
    for (int j = 0; j < K; ++j) L.pos[j] = (uint32_t)L.id[j] < (uint32_t)bv.m ? pv.inv[L.id[j]] : -1;
    done = L.pos[K - 1] >= 0;
  }
  if (!done) {  // the BVH search, compacted into k_normals_queue (a wave here
    // would wait on its slowest lane's search: r10g, 0.72 ms a frame),
    // capped by the seeds' K-th distance (no point beyond it can be among
    // the K nearest: r10g, uncapped, ~1 ms for a few thousand points)
    const int at = atomicAdd(fbq, 1);
    fbq[2 + 2 * at] = pos;
    fbq[3 + 2 * at] = __float_as_int(L.bound());
    return;
  }
  nrm[pos] = knn_normal<K>(bv, L, p, vx, vy, vz);
}

// The K nearest within d2 <= cap (the caller knows K points within it, so
// the K nearest are among them): the BVH walk prunes every box beyond it.
template <int K>
struct BestKCap {
  BestK<K> L;
  float cap;
  RST_HD float bound() const { return fminf(cap, L.bound()); }
  RST_HD void offer(float nd, int nid, int np) {
    if (nd <= cap) L.offer(nd, nid, np);
  }
};

// The grid search's leftovers (~0.7% of a 640x480 frame: oblique surfaces
// whose 7 x 7 seeds' K-th distance maps to a window just wider than the
// staged halo -- median 10 pixels, the true K-th's 6), one wavefront each:
// the window of the cap (<= kNwHalf pixels) scanned from global memory, 64
// pixels a lane round, the candidates within the bound appended to an LDS
// list; a list near full is cut to its K smallest (rank by counting,
// ties by original index as BestK), which tightens the bound.  A cap whose
// window is wider first scans the kNwProbe box around the point's pixel for
// a bound.  Windows beyond that (isolated points: a few a frame) take lane
// 0's BVH search, capped.  Same (d2, index) order, so the same K and the
// same normal as k_normals.  r10h: the per-lane BVH search of the same
// queue took 0.85 ms (its slowest lanes).
#ifndef RST_KNN_WAVE
#define RST_KNN_WAVE 1  // 0: the leftovers' per-lane BVH search (k_normals_queue)
#endif
constexpr int kNwCap = 192;  // list entries per wavefront (cut at > kNwCap - 64)
constexpr int kNwHalf = 32;   // widest window scanned (pixels)
constexpr int kNwProbe = 12;  // the probe box's half side (pixels)
constexpr int kNwWaves = 4;

template <int K>
struct NwList {
  float d[kNwCap];
  int id[kNwCap];
  float td[K];
  int tid[K];
};

// cut the list to its K smallest (d, id), sorted; returns the new length
template <int K>
__device__ __forceinline__ int nw_select(NwList<K>& s, int n, int lane) {
  for (int c = lane; c < n; c += kWave) {
    const float dc = s.d[c];
    const int ic = s.id[c];
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += lex_less(s.d[j], s.id[j], dc, ic) ? 1 : 0;
    if (rank < K) {
      s.td[rank] = dc;
      s.tid[rank] = ic;
    }
  }
  wave_sync();
  const int nk = min(n, K);
  if (lane < nk) {
    s.d[lane] = s.td[lane];
    s.id[lane] = s.tid[lane];
  }
  wave_sync();
  return nk;
}

// the pixels [a0, a1] x [b0, b1] into the list (candidates d2 <= *bound)
template <int K>
__device__ __forceinline__ int nw_scan(const PixView& pv, const float4& p, int a0, int a1, int b0, int b1,
                                       NwList<K>& s, int n, float* bound, int lane) {
  const int ww = a1 - a0 + 1, np = ww * (b1 - b0 + 1);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int base = 0; base < np; base += 4 * kWave) {
    float4 t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // four loads in flight per lane
      const int k = base + j * kWave + lane;
      t[j] = k < np ? pv.pts[(int64_t)(b0 + k / ww) * pv.w + (a0 + k % ww)] : make_float4(NAN, NAN, NAN, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = d2_ref(p.x, p.y, p.z, t[j].x, t[j].y, t[j].z);  // (NaN: no point)
      const bool in = d <= *bound;
      const uint64_t m = __ballot(in);
      if (in) {
        const int at = n + __popcll(m & lt);
        s.d[at] = d;
        s.id[at] = f2i(t[j].w);
      }
      n += __popcll(m);
      if (n > kNwCap - kWave) {  // (uniform)
        wave_sync();
        n = nw_select<K>(s, n, lane);
        if (n == K) *bound = s.d[K - 1];
      }
    }
  }
  wave_sync();
  return n;
}

template <int K>
__global__ __launch_bounds__(kWave* kNwWaves) void k_normals_wave(BvhView bv, PixView pv,
                                                                   const int32_t* __restrict__ fbq, float vx,
                                                                   float vy, float vz,
                                                                   float4* __restrict__ nrm) {
  __shared__ NwList<K> lists[kNwWaves];
  const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  NwList<K>& s = lists[w];
  const int nq = fbq[0];
  for (int j = blockIdx.x * kNwWaves + w; j < nq; j += gridDim.x * kNwWaves) {
    const int pos = fbq[2 + 2 * j];
    if ((uint32_t)pos >= (uint32_t)bv.m) continue;  // (uniform)
    const float4 p = bv.pts[pos];
    float bound = __int_as_float(fbq[3 + 2 * j]);  // K points lie within it (FLT_MAX: unknown)
    int a0, a1, b0, b1;
    float rc;
    bool win = pix_window(pv, p.x, p.y, p.z, bound, (float)kNwHalf, a0, a1, b0, b1, rc);
    if (!win && p.z > 0.f) {  // a bound from the probe box
      const float iz = 1.0f / p.z;
      const int uc = (int)floorf((pv.fx * p.x * iz + pv.cx) / (float)pv.s + 0.5f);
      const int vc = (int)floorf((pv.fy * p.y * iz + pv.cy) / (float)pv.s + 0.5f);
      const int pa0 = max(0, uc - kNwProbe), pa1 = min(pv.w - 1, uc + kNwProbe);
      const int pb0 = max(0, vc - kNwProbe), pb1 = min(pv.h - 1, vc + kNwProbe);
      if (pa0 <= pa1 && pb0 <= pb1) {
        const int n = nw_scan<K>(pv, p, pa0, pa1, pb0, pb1, s, 0, &bound, lane);
        if (n >= K) {
          nw_select<K>(s, n, lane);
          bound = s.d[K - 1];
        }
        win = pix_window(pv, p.x, p.y, p.z, bound, (float)kNwHalf, a0, a1, b0, b1, rc);
      }
    }
    bool done = false;
    if (win) {
      int n = nw_scan<K>(pv, p, a0, a1, b0, b1, s, 0, &bound, lane);
      if (n >= K) {
        n = nw_select<K>(s, n, lane);
        done = margin_sqrt(s.d[K - 1]) * 1.00001f + 1e-30f < rc;
      }
    }
    if (lane == 0) {
      BestK<K> L;
      if (done) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          L.d[k] = s.d[k];
          L.id[k] = s.id[k];
          L.pos[k] = (uint32_t)s.id[k] < (uint32_t)bv.m ? pv.inv[s.id[k]] : -1;
        }
        done = L.pos[K - 1] >= 0;
      }
      if (!done) {
        BestKCap<K> R;
        R.L.init();
        R.cap = __int_as_float(fbq[3 + 2 * j]);
        search(bv, pos, p.x, p.y, p.z, R);
        L = R.L;
      }
      nrm[pos] = knn_normal<K>(bv, L, p, vx, vy, vz);
    }
    wave_sync();
  }
}

// the grid search's leftovers: the BVH search from the point's own leaf
template <int K>
__global__ __launch_bounds__(kBS) void k_normals_queue(BvhView bv, const int32_t* __restrict__ fbq, float vx,
                                                       float vy, float vz, float4* __restrict__ nrm) {
  const int j = blockIdx.x * kBS + threadIdx.x;
  if (j >= fbq[0]) return;
  const int pos = fbq[2 + 2 * j];
  if ((uint32_t)pos >= (uint32_t)bv.m) return;
  const float4 p = bv.pts[pos];
  BestKCap<K> R;
  R.L.init();
  R.cap = __int_as_float(fbq[3 + 2 * j]);  // (FLT_MAX: fewer than K seeds)
  search(bv, pos, p.x, p.y, p.z, R);
  nrm[pos] = knn_normal<K>(bv, R.L, p, vx, vy, vz);
}

// Image-grid normals (the point-to-plane perf mode; the reference's
// ComputeNormals, point_cloud_utils.cpp:176-204, finds its 16 neighbours by
// kNN -- a frame target already has them on its pixel grid).  A 16 x 16
// block of level pixels stages its (16 + 2r)^2 window of points in LDS (map
// -> sorted position -> point); each valid pixel takes the window points
// within kGridReach window-pitches of itself (depth edges excluded), and
// their fp32 centroid / covariance PCA (as the reference's, in window order)
// gives the normal, oriented as OrientNormals (:206-216).  Fewer than 3
// points: the normal faces the viewpoint.  12 B map/pt in, 16 B/pt out.
constexpr int kGridT = 16;
constexpr int kGridMaxR = 2;
constexpr float kGridReach = 5.0f;  // allows surfaces ~78 deg from the image plane

__global__ __launch_bounds__(kGridT* kGridT) void k_grid_normals(PixView pv, const float4* __restrict__ pts,
                                                                int r, float vx, float vy, float vz,
                                                                float4* __restrict__ nrm) {
  constexpr int TW = kGridT + 2 * kGridMaxR;
  __shared__ float4 tile[TW * TW];
  const int tw = kGridT + 2 * r;
  const int u0 = blockIdx.x * kGridT - r, v0 = blockIdx.y * kGridT - r;
  for (int k = threadIdx.x; k < tw * tw; k += kGridT * kGridT) {
    const int uu = u0 + k % tw, vv = v0 + k / tw;
    int pos = -1;
    if (uu >= 0 && vv >= 0 && uu < pv.w && vv < pv.h) pos = pv.map[(int64_t)vv * pv.w + uu];
    tile[k] = pos >= 0 ? pts[pos] : make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
  }
  __syncthreads();
  const int lu = threadIdx.x % kGridT, lv = threadIdx.x / kGridT;
  const int u = blockIdx.x * kGridT + lu, v = blockIdx.y * kGridT + lv;
  if (u >= pv.w || v >= pv.h) return;
  const int pos = pv.map[(int64_t)v * pv.w + u];
  if (pos < 0) return;
  const float4 p = tile[(lv + r) * tw + (lu + r)];
  // window pitch at this depth: pixel spacing s z / fx, r of them
  const float reach = kGridReach * (float)(r > 0 ? r : 1) * (float)pv.s * p.z / fabsf(pv.fx);
  const float reach2 = reach * reach;
  int cnt = 0;
  float cx = 0.f, cy = 0.f, cz = 0.f;
  for (int dv = 0; dv <= 2 * r; ++dv)
    for (int du = 0; du <= 2 * r; ++du) {
      const float4 q = tile[(lv + dv) * tw + (lu + du)];
      if (__float_as_int(q.w) < 0) continue;
      const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
      if ((dx * dx + dy * dy) + dz * dz > reach2) continue;
      cx += q.x;
      cy += q.y;
      cz += q.z;
      ++cnt;
    }
  float nx, ny, nz;
  if (cnt >= 3) {
    const float kf = (float)cnt;
    cx = cx / kf;
    cy = cy / kf;
    cz = cz / kf;
    float c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
    for (int dv = 0; dv <= 2 * r; ++dv)
      for (int du = 0; du <= 2 * r; ++du) {
        const float4 q = tile[(lv + dv) * tw + (lu + du)];
        if (__float_as_int(q.w) < 0) continue;
        const float ex = q.x - p.x, ey = q.y - p.y, ez = q.z - p.z;
        if ((ex * ex + ey * ey) + ez * ez > reach2) continue;
        const float dx = q.x - cx, dy = q.y - cy, dz = q.z - cz;
        c00 += dx * dx; c01 += dx * dy; c02 += dx * dz;
        c11 += dy * dy; c12 += dy * dz; c22 += dz * dz;
      }
    const double a[6] = {c00, c01, c02, c11, c12, c22};
    double e[3];
    sym3_min_vec(a, e);
    nx = (float)e[0];
    ny = (float)e[1];
    nz = (float)e[2];
  } else {
    nx = p.x - vx;
    ny = p.y - vy;
    nz = p.z - vz;
    const float l = sqrtf((nx * nx + ny * ny) + nz * nz);
    const float il = l > 0.f ? 1.0f / l : 0.f;
    nx *= il;
    ny *= il;
    nz = l > 0.f ? nz * il : 1.f;
  }
  const float rx = p.x - vx, ry = p.y - vy, rz = p.z - vz;
  if (rx * nx + (ry * ny + rz * nz) > 0) {  // OrientNormals
    nx = -nx;
    ny = -ny;
    nz = -nz;
  }
  nrm[pos] = make_float4(nx, ny, nz, 0.0f);
}

inline int blocks_for(int64_t n) { return (int)std::max<int64_t>(1, (n + kBS - 1) / kBS); }

}  // namespace

int query_nn_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q, int64_t nq,
                    int32_t* d_idx, float* d_d2) {
  if (!ctx || !tgt || nq < 0 || !tgt->has_bvh) return RST_E_ARG;
  if (nq == 0) return RST_OK;
  if (tgt->m == 0) {
    // empty index: nothing is ever added -> (0, FLT_MAX)
    RST_HIP(hipMemsetAsync(d_idx, 0, sizeof(int32_t) * nq, ctx->stream));
    std::vector<float> f(nq, FLT_MAX);
    RST_HIP(hipMemcpyAsync(d_d2, f.data(), sizeof(float) * nq, hipMemcpyHostToDevice,
                           ctx->stream));
    RST_HIP(hipStreamSynchronize(ctx->stream));
    return RST_OK;
  }
  k_query_nn<<<blocks_for(nq), kBS, 0, ctx->stream>>>(view_of(tgt), d_q, nq, d_idx, d_d2);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int query_nn_warm_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q, int64_t nq,
                         const int32_t* d_warm, int32_t* d_idx, float* d_d2, int* d_stats) {
  if (!ctx || !tgt || nq < 0 || !tgt->has_bvh) return RST_E_ARG;
  if (nq == 0) return RST_OK;
  if (tgt->m == 0) return query_nn_device(ctx, tgt, d_q, nq, d_idx, d_d2);
  k_query_nn_warm<<<blocks_for(nq), kBS, 0, ctx->stream>>>(view_of(tgt), tgt->inv, d_q, nq, d_warm,
                                                           d_idx, d_d2, d_stats);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int query_nn_fallback_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q, int64_t nq,
                             const int32_t* d_warm, int mode, int32_t* d_idx, float* d_d2,
                             int32_t* d_path) {
  if (!ctx || !tgt || nq < 0 || !tgt->has_bvh) return RST_E_ARG;
  if (nq == 0) return RST_OK;
  const int64_t nb = (nq + kBS / kWave - 1) / (kBS / kWave);
  k_query_nn_fallback<<<(unsigned)nb, kBS, 0, ctx->stream>>>(view_of(tgt), adj_of(tgt), tgt->inv,
                                                             d_q, nq, d_warm, mode, d_idx, d_d2,
                                                             d_path);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int query_knn_device(rst_ctx* ctx, const rst_target* tgt, const float* d_q, int64_t nq,
                     int k, int32_t* d_idx, float* d_d2) {
  if (!ctx || !tgt || nq < 0 || k < 1 || k > 32 || !tgt->has_bvh || tgt->m == 0)
    return RST_E_ARG;
  if (nq == 0) return RST_OK;
  const BvhView v = view_of(tgt);
  hipStream_t st = ctx->stream;
  if (k <= 1)
    k_query_knn<1><<<blocks_for(nq), kBS, 0, st>>>(v, d_q, nq, k, d_idx, d_d2);
  else if (k <= 4)
    k_query_knn<4><<<blocks_for(nq), kBS, 0, st>>>(v, d_q, nq, k, d_idx, d_d2);
  else if (k <= 8)
    k_query_knn<8><<<blocks_for(nq), kBS, 0, st>>>(v, d_q, nq, k, d_idx, d_d2);
  else if (k <= 16)
    k_query_knn<16><<<blocks_for(nq), kBS, 0, st>>>(v, d_q, nq, k, d_idx, d_d2);
  else
    k_query_knn<32><<<blocks_for(nq), kBS, 0, st>>>(v, d_q, nq, k, d_idx, d_d2);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int compute_normals(rst_ctx* ctx, rst_target* tgt, int k, const float vp[3]) {
  if (!ctx || !tgt || !tgt->has_bvh) return RST_E_ARG;
  if (k != 8 && k != 16 && k != 32) return RST_E_ARG;  // compiled K values
  // m < k would leave result slots at the reference's idx 0 default
  // (std::vector<int> oi(k) zero-initialised); not supported here
  if (tgt->m < k) return RST_E_ARG;
  if (!tgt->nrm) {
    if (target_alloc(tgt, sizeof(float4) * std::max<int64_t>(tgt->m, 1), (void**)&tgt->nrm) < 0)
      return RST_E_NOMEM;
  }
  if (tgt->m == 0) return RST_OK;
  const BvhView v = view_of(tgt);
  hipStream_t st = ctx->stream;
  const float x = vp ? vp[0] : 0.f, y = vp ? vp[1] : 0.f, z = vp ? vp[2] : 0.f;
  // frame targets: the pixel grid's windows (RST_KNN_GRID=0: the BVH search)
  static const bool grid_ok = [] {
    const char* e = getenv("RST_KNN_GRID");
    return !e || atoi(e) != 0;
  }();
  if (tgt->pix.map && grid_ok && k == 16) {
    int32_t* fbq = nullptr;  // [count, positions...]
    RST_CHECK(ctx_workspace(ctx, sizeof(int32_t) * (2 * (size_t)tgt->m + 64), (void**)&fbq));
    RST_HIP(hipMemsetAsync(fbq, 0, sizeof(int32_t), st));
    k_normals_grid<16><<<dim3((tgt->pix.w + kKnnT - 1) / kKnnT, (tgt->pix.h + kKnnT - 1) / kKnnT),
                         kKnnT * kKnnT, 0, st>>>(v, tgt->pix, x, y, z, tgt->nrm, fbq);
#if RST_KNN_WAVE
    k_normals_wave<16><<<512, kWave * kNwWaves, 0, st>>>(v, tgt->pix, fbq, x, y, z, tgt->nrm);
#else
    k_normals_queue<16><<<blocks_for(tgt->m), kBS, 0, st>>>(v, fbq, x, y, z, tgt->nrm);
#endif
  } else if (k == 8)
    k_normals<8><<<blocks_for(tgt->m), kBS, 0, st>>>(v, tgt->m, x, y, z, tgt->nrm);
  else if (k == 16)
    k_normals<16><<<blocks_for(tgt->m), kBS, 0, st>>>(v, tgt->m, x, y, z, tgt->nrm);
  else
    k_normals<32><<<blocks_for(tgt->m), kBS, 0, st>>>(v, tgt->m, x, y, z, tgt->nrm);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int compute_grid_normals(rst_ctx* ctx, rst_target* tgt, int r, const float vp[3]) {
  if (!ctx || !tgt) return RST_E_ARG;
  if (r < 1 || r > kGridMaxR) return RST_E_ARG;
  if (!tgt->pix.map) return RST_E_STATE;  // not prepared from a depth frame
  if (!tgt->nrm) {
    if (target_alloc(tgt, sizeof(float4) * std::max<int64_t>(tgt->m, 1), (void**)&tgt->nrm) < 0)
      return RST_E_NOMEM;
  }
  if (tgt->m == 0) return RST_OK;
  const float x = vp ? vp[0] : 0.f, y = vp ? vp[1] : 0.f, z = vp ? vp[2] : 0.f;
  const dim3 grid((tgt->pix.w + kGridT - 1) / kGridT, (tgt->pix.h + kGridT - 1) / kGridT);
  k_grid_normals<<<grid, kGridT * kGridT, 0, ctx->stream>>>(tgt->pix, tgt->pts, r, x, y, z,
                                                            tgt->nrm);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

}  // namespace rst
