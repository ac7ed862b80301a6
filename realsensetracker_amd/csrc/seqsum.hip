// seqsum.hip -- the reference's sequential float32 sums, computed in parallel
// and bit-exact.
//
// RST_SUM_REF replays `dst_mean += dst.GetPoint(j)` / `cost += dist_sqr`
// (align_icp.cpp:113,120) and ComputeCentroid's loop
// (point_cloud_utils.cpp:94-96): s_{k+1} = fl(s_k + x_k) in float32,
// round-to-nearest-even, k ascending from s_0 = +0.  One wavefront replaying
// the chain (k_seq_sum4 in icp.hip) takes ~1.4 ms at 300k points.  Here the
// chain is cut into stretches whose maps (rst_seqsum.hpp: the offset rule,
// verified windows, residue candidates) are built in parallel, composed in
// two levels, and walked by one wavefront in a few dozen verified jumps.
//
// Per chain c (one float component of a float4 stream x[0..n)):
//   k_sq_tot    per 4096-element tile: the SoA copy, fp64 tile total,
//               non-finite flags per 16-element window;
//   k_sq_guess  per tile: the fp64 prefix of every element (an APPROXIMATE
//               start, only to place boundaries and seed guesses); block
//               starts = the element of largest |prefix| in each 16-element
//               window, group starts = the block of largest |prefix| in each
//               16-block window, a superblock start per tile likewise (maps
//               start where the sum is large: their grids then bound every
//               grid inside, so few residue candidates cover them); each
//               block's unmonitored float32 run from its fp64 guess -> its
//               increment;
//   k_sq_maps   per superblock: the drift-corrected guesses (the fp64
//               prefix of the blocks' float32 increments: within a few ulps
//               of the true sums, where the fp64 prefix can be thousands of
//               ulps off), then per block its monitored runs from 4
//               candidates (leaf maps), per group the composite of its
//               blocks for up to 16 candidates, per superblock the composite
//               of its groups for up to 64 candidates;
//   k_sq_walk   one wavefront per chain: s = +0; per superblock one verified
//               jump (residue, window, E + d); a failed check descends to the
//               superblock's group maps, then leaf maps, then the block's
//               own float adds.  inf/NaN short-circuit through the flags.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "rst_device.hpp"
#include "rst_internal.hpp"
#include "rst_seqsum.hpp"

namespace rst {
namespace {

using namespace sq;

struct SqView {
  int64_t n;
  int64_t ns;      // SoA row stride (n rounded up to 64)
  int nch;
  int nb, ng, nk;  // blocks, groups, superblocks (= tiles)
  float* soa;      // [nch][ns]
  uint8_t* wflg;   // [nch][nb]: 1 NaN, 2 +inf, 4 -inf in the block window
  int* bs;         // [nch][nb + 1]
  int* gs;         // [nch][ng + 1]
  int* ks;         // [nch][nk + 1]
  double* inc;     // [nch][nb]
  double* ipre;    // [nch][nb]: exclusive prefix of inc within the block's tile
  double* tinc;    // [nch][nk]
  Leaf* leaf;      // [nch][nb]
  GroupMap* grp;   // [nch][ng]
  SbMap* sbm;      // [nch][nk]
  int* stats;      // optional, 8 per chain
  double* ttot;    // [nch][4 nk] fp64 totals of 1024-element quarter tiles (this call's)
  double* ttot2;   // [2][4][4 nk] the same, by iteration parity (the fused front
                   // reads the previous iteration's, writes its own)
  long long* clk;  // [nch][nk][8] shader clocks at the map kernel's phase boundaries
  int* err;        // bound-check failures (bits; 0 = none): a map kernel that
                   // meets a size its tables cannot hold stops instead of
                   // reading out of range
  // a stretch of a longer chain (the sharded loop's relay, comm.hip): per
  // chain the fp64 prefix before the stretch (the guesses' offset) and the
  // chain's value where it starts (the walk's start); null = a whole chain
  const double* p0;
  const float* s0;
  unsigned long long* tl;  // RST_TIMELINE builds: the ICP loop's kernel timeline
  int it;                  // ... and this iteration
  int* guard;              // optional: the ICP state's guard word -- a tripped bound
                           // check (err) reaches the align's result as an
                           // internal error, not as the reference's false
};

// diagnostics (rst_debug_seqsum_fault): bits OR-ed into err by every walk,
// so a test can trip the guard path without corrupting a table
__device__ int g_sq_fault = 0;

__device__ __forceinline__ float comp(const float4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ int nf_flags(float x) {
  if (isnan(x)) return 1;
  if (isinf(x)) return x > 0 ? 2 : 4;
  return 0;
}

// a double through a DPP lane move (both halves; lanes without a source,
// or outside row_mask, get +0)
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp_d(double x) {
  const uint2 u = __builtin_bit_cast(uint2, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u.x, CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)u.y, CTRL, ROWS, 0xf, false);
  return __builtin_bit_cast(double, make_uint2((unsigned)lo, (unsigned)hi));
}
// inclusive scan of one double per lane over the wave, all by DPP (no LDS):
// Hillis-Steele inside each row of 16 (row_shr 1, 2, 4, 8), then row 15's
// total into rows 1 and 3 (row_bcast15) and lane 31's into rows 2 and 3
// (row_bcast31).  The whole wave must be active.  (Its additions associate
// differently from a serial sum: its users take these fp64 prefixes as
// guesses only -- block starts, map candidates -- never as results.)
__device__ __forceinline__ double wave_scan_incl(double x) {
  x += dpp_d<0x111>(x);  // row_shr:1
  x += dpp_d<0x112>(x);  // row_shr:2
  x += dpp_d<0x114>(x);  // row_shr:4
  x += dpp_d<0x118>(x);  // row_shr:8
  x += dpp_d<0x142, 0xa>(x);  // row_bcast:15 -> rows 1, 3
  x += dpp_d<0x143, 0xc>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}

// a lane's value from a DPP partner (int)
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
// the DPP partners of a 16-lane row butterfly: quad_perm [1,0,3,2] and
// [2,3,0,1] (lane ^ 1, ^ 2), then row_half_mirror and row_mirror, whose
// partners stand for ^ 4 and ^ 8 once the quads and the half rows agree --
// valid for an associative, commutative, order-free merge (min, max, a
// lexicographic max), not for sums (r22: in place of ds_bpermute steps)
constexpr int kRowBfly[4] = {0xB1, 0x4E, 0x141, 0x140};
// lane 0's double, as a scalar
__device__ __forceinline__ double rd_lane0(double x) {
  const uint2 u = __builtin_bit_cast(uint2, x);
  return __builtin_bit_cast(double, make_uint2((unsigned)__builtin_amdgcn_readlane((int)u.x, 0),
                                               (unsigned)__builtin_amdgcn_readlane((int)u.y, 0)));
}
// the whole wave's fp64 sum (a guess's: its association is the scan's) at
// lane kWave - 1
__device__ __forceinline__ double wave_sum_last(double x) { return wave_scan_incl(x); }

// exclusive block scan of one double per thread (BS threads); returns the
// prefix, *total = the block total
// (r19: DPP scans instead of a ds_bpermute per step and thread 0's serial
// pass over the waves' totals -- the guesses' prefixes only, see above)
template <int BS>
__device__ double block_scan_excl(double v, double* lds, double* total) {
  constexpr int NW = BS / kWave;
  static_assert(NW <= kWave, "one wave scans the waves' totals");
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const double inc = wave_scan_incl(v);
  if (lane == kWave - 1) lds[w] = inc;
  __syncthreads();
  if (w == 0) {
    const double t = lane < NW ? lds[lane] : 0.0;
    const double ti = wave_scan_incl(t);
    if (lane < NW) lds[lane] = ti - t;
    if (lane == NW - 1) lds[NW] = ti;
  }
  __syncthreads();
  const double r = lds[w] + inc - v;
  *total = lds[NW];
  __syncthreads();
  return r;
}

// sum of a[0..cnt) (doubles, global) over the block, fixed order per thread
template <int BS>
__device__ double block_sum_global(const double* a, int cnt, double* lds) {
  double s = 0.0;
  // (four loads in flight per round: a rolled loop waited one trip each)
  for (int i0 = threadIdx.x; i0 < cnt; i0 += 4 * BS) {
    double t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = i0 + u * BS < cnt ? a[i0 + u * BS] : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) s += t[u];
  }
  double tot;
  (void)block_scan_excl<BS>(s, lds, &tot);
  return tot;
}

// ---- 0: small streams, the chains replayed ----------------------------------------
// Below RST_SQ_SERIAL_MAX elements the map pipeline's five dependent
// launches (~50 us of fixed latency however short the stream) cost more
// than replaying the chains: lane c < 4 carries chain c through s = fl(s + x_i), i
// ascending from +0 -- the reference's loop itself, so inf / NaN / subnormal
// need no case analysis -- one dependent v_add_f32 per element.  The
// wavefront only keeps it fed: tiles of 64 x kSerT float4 loaded coalesced
// a tile ahead, transposed through LDS so lane c reads four of its values
// per ds_read_b128, kSerG reads in flight ahead of the adds.  A tile's tail
// past n is +0: s is never -0 (from +0, fl(a + b) = -0 needs a = b = -0),
// so fl(s + 0) = s and the padded adds change no bit.
constexpr int kSerT = 16;                   // float4 per lane per tile (1024 elements)
constexpr int kSerRow = kSerT * kWave + 4;  // floats per chain row (+4: rows on distinct banks)
constexpr int kSerG = 8;                    // ds_read_b128 per group (32 elements)
// RST_SQ_SERIAL_MAX default.  A lone wavefront's dependent v_add_f32 costs
// ~12 clocks (the ISA is 32 back-to-back adds per group): 5.0 ns an element
// against the pipeline's ~53 us flat (r05a, tools/seq_serial_sweep.py:
// 2k / 4k / 8k / 15k / 33k elements 13 / 23 / 43 / 77 / 163 us replayed vs
// 64 / 50 / 55 / 53 / 53 us mapped) -- the callers' ~15k-point clouds stay
// on the pipeline
constexpr int kSerDefault = 8192;

__device__ __forceinline__ void ser_load(const float4* __restrict__ x, int64_t n, int64_t base,
                                         float4 (&v)[kSerT]) {
#pragma unroll
  for (int t = 0; t < kSerT; ++t) {
    const int64_t i = base + (int64_t)t * kWave + threadIdx.x;
    v[t] = i < n ? x[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

__device__ __forceinline__ void ser_group(const float* row, float4 (&q)[kSerG]) {
#pragma unroll
  for (int k = 0; k < kSerG; ++k) q[k] = *reinterpret_cast<const float4*>(row + 4 * k);
}

__device__ __forceinline__ void ser_add(const float4 (&q)[kSerG], float& s) {
#pragma unroll
  for (int k = 0; k < kSerG; ++k) {
    s = s + q[k].x;
    s = s + q[k].y;
    s = s + q[k].z;
    s = s + q[k].w;
  }
}

// one tile: transpose, then lane c's chain over its first cnt values
// (rounded up to a group: the rest are +0)
__device__ __forceinline__ void ser_tile(const float4 (&v)[kSerT], int cnt, float* tile, float& s) {
  const int lane = threadIdx.x;
  __syncthreads();  // (the previous tile's reads are done)
#pragma unroll
  for (int t = 0; t < kSerT; ++t) {
    tile[0 * kSerRow + t * kWave + lane] = v[t].x;
    tile[1 * kSerRow + t * kWave + lane] = v[t].y;
    tile[2 * kSerRow + t * kWave + lane] = v[t].z;
    tile[3 * kSerRow + t * kWave + lane] = v[t].w;
  }
  __syncthreads();
  if (lane < 4) {
    const float* row = tile + lane * kSerRow;
    constexpr int kGE = 4 * kSerG;  // elements per group
    const int ng = (cnt + kGE - 1) / kGE;
    float4 q[kSerG], r[kSerG];
    ser_group(row, q);
    int g = 0;
    // two groups per trip: one group's reads in flight during the other's adds
    for (; g + 2 <= ng; g += 2) {
      ser_group(row + (g + 1) * kGE, r);
      ser_add(q, s);
      if (g + 2 < ng) ser_group(row + (g + 2) * kGE, q);
      ser_add(r, s);
    }
    if (g < ng) ser_add(q, s);
  }
}

__global__ __launch_bounds__(kWave) void k_sq_serial(const float4* __restrict__ x, int64_t n, int nch,
                                                     const float* __restrict__ s0, float* __restrict__ out) {
  __shared__ float4 tile4[kSerRow];  // 4 rows of kSerRow floats
  float* tile = reinterpret_cast<float*>(tile4);
  constexpr int64_t kT = (int64_t)kSerT * kWave;
  float s = s0 && (int)threadIdx.x < nch ? s0[threadIdx.x] : 0.0f;
  float4 a[kSerT], b[kSerT];
  ser_load(x, n, 0, a);
  for (int64_t base = 0; base < n; base += 2 * kT) {
    ser_load(x, n, base + kT, b);  // in flight during a's chain
    ser_tile(a, (int)min<int64_t>(n - base, kT), tile, s);
    if (base + kT >= n) break;
    ser_load(x, n, base + 2 * kT, a);
    ser_tile(b, (int)min<int64_t>(n - base - kT, kT), tile, s);
  }
  if ((int)threadIdx.x < nch) out[threadIdx.x] = s;
}

// ---- 1: SoA copy, window flags, fp64 totals --------------------------------------
// One 1024-element quarter tile per workgroup, four consecutive elements
// per thread (64 contiguous bytes: coalesced float4 loads, one float4 SoA
// store per component); a 16-element window is a lane quad, its flags
// OR-ed across the quad by DPP.  The quarter tile's fp64 total per
// component: the threads' 4-element sums (fixed order), reduced over the
// block (fixed tree) -- four components in one reduction.
constexpr int kFrontT = kTile / kW;  // 256

constexpr int kTotE = 1024;          // elements per k_sq_tot workgroup
constexpr int kTotQ = kTile / kTotE; // 4 per tile
static_assert(kTotE == 4 * kFrontT, "k_sq_tot: four elements per thread");

// quad_perm DPP: lane ^ 1 and lane ^ 2 within each lane quad
__device__ __forceinline__ int quad_or(int a) {
  a |= __builtin_amdgcn_mov_dpp(a, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  a |= __builtin_amdgcn_mov_dpp(a, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  return a;
}

__device__ __forceinline__ void sq_tot_body(const float4* __restrict__ x, const SqView& v, const int qt) {
  RST_TL(v.tl, v.it, 2);
  __shared__ double red[kFrontT / kWave][4];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  const int64_t i0 = (int64_t)qt * kTotE + 4 * tid;
  float4 q[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = i0 + j < v.n ? x[i0 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
  double part[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float e[4];
    int f = 0;
    double ps = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      e[j] = comp(q[j], c);
      const int fj = nf_flags(e[j]);
      f |= fj;
      ps += fj ? 0.0 : (double)e[j];
    }
    part[c] = ps;
    if (c < v.nch) {
      float* dst = v.soa + (int64_t)c * v.ns;
      // (ns is a multiple of 64 and i0 of 4: the float4 is in the row)
      if (i0 < v.n) *reinterpret_cast<float4*>(dst + i0) = make_float4(e[0], e[1], e[2], e[3]);
      f = quad_or(f);
      const int64_t w = i0 / kW;
      if ((tid & 3) == 0 && w < v.nb) v.wflg[(int64_t)c * v.nb + w] = (uint8_t)f;
    }
  }
  // (the wave's totals by DPP scans -- fp64 guesses, any association;
  // r22: a ds_bpermute butterfly, 48 LDS round trips a wavefront)
#pragma unroll
  for (int c = 0; c < 4; ++c) part[c] = wave_sum_last(part[c]);
  if (lane == kWave - 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) red[wv][c] = part[c];
  __syncthreads();
  if (tid < v.nch) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kFrontT / kWave; ++w) t += red[w][tid];
    v.ttot[(int64_t)tid * v.nk * kTotQ + qt] = t;
  }
}

// ---- 2: boundaries, unmonitored runs, increments ----------------------------------
// One workgroup per (tile, chain); thread = one 16-element window.
// FUSED (an ICP iteration after the first, the same chains as the one
// before): no k_sq_tot launch -- the tile comes straight from the float4
// stream, the SoA row, window flags and quarter totals are written here, and
// the tile prefix P is the PREVIOUS iteration's (P only places the block
// boundaries and seeds the guesses: a stale P costs map hits, never a bit
// of the result).
template <bool FUSED>
__device__ __forceinline__ void sq_front_body(const SqView& v, const float4* __restrict__ x,
                                              const double* __restrict__ tprev, double* __restrict__ tnext,
                                              const int t, const int c) {
  RST_TL(v.tl, v.it, 3);
  // (one pad float per 16: thread t's window reads xs(16 t + j) at 17 t + j,
  // every lane in its own bank)
  __shared__ float xsp[(kTile + kW) + (kTile + kW) / kW];
  auto xs = [&](int i) -> float& { return xsp[i + (i >> 4)]; };
  __shared__ int sbs[kFrontT + 1];
  __shared__ double sA[kFrontT];
  __shared__ double lds[kFrontT / kWave + 1];
  __shared__ double gkey[kKW];
  __shared__ int gid[kKW];
  const int tid = threadIdx.x;
  const int64_t e0 = (int64_t)t * kTile;
  if (t == 0 && c == 0 && tid == 0) *v.err = 0;
  // the tile (and the next tile's first window) of component c
  const float* Xs = v.soa + (int64_t)c * v.ns;
  double P;
  {
    // (every load issued before the first LDS store: a rolled loop waited
    // out one memory round trip per element)
    constexpr int kJ = (kTile + kW + kFrontT - 1) / kFrontT;
    float tv[kJ];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const int i = tid + j * kFrontT;
      if (FUSED)
        tv[j] = i < kTile + kW && e0 + i < v.n ? comp(x[e0 + i], c) : 0.0f;
      else
        tv[j] = i < kTile + kW && e0 + i < v.n ? Xs[e0 + i] : 0.0f;
    }
    // fp64 prefix at the tile start (the quarter tiles' totals before it;
    // r22: its loads in flight with the tile's, one memory trip, not two)
    P = block_sum_global<kFrontT>((FUSED ? tprev : v.ttot) + (int64_t)c * v.nk * kTotQ, t * kTotQ, lds) +
        (v.p0 ? v.p0[c] : 0.0);
    if (FUSED) {
      float* dst = v.soa + (int64_t)c * v.ns;
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const int i = tid + j * kFrontT;
        if (i < kTile && e0 + i < v.n) dst[e0 + i] = tv[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const int i = tid + j * kFrontT;
      if (i < kTile + kW) xs(i) = tv[j];
    }
  }
  __syncthreads();
  // the thread's window: fp64 total and prefix
  const int b = t * kBlocksPerTile + tid;
  double wsum = 0.0;
  int wfl = 0;
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    const float e = xs(tid * kW + j);
    wfl |= nf_flags(e);
    if (isfinite(e)) wsum += (double)e;
  }
  if (FUSED) {
    // the window's non-finite flags and this iteration's quarter totals (one
    // quarter per wavefront: 64 windows of 16)
    if (b < v.nb) v.wflg[(int64_t)c * v.nb + b] = (uint8_t)wfl;
    double q = wsum;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, kWave);
    if ((tid & (kWave - 1)) == 0) tnext[(int64_t)c * v.nk * kTotQ + t * kTotQ + tid / kWave] = q;
  }
  double ttotal;
  const double wrel = block_scan_excl<kFrontT>(wsum, lds, &ttotal);
  // block start: the element of largest |prefix| among positions
  // [kJLo, kJHi] of the window (the prefix before the element: the value a
  // block starting there starts from); the middle of the window only, so
  // block, group and superblock sizes stay within ~1.5x of the mean (the
  // map kernel's time follows its largest superblock and group)
  const double wpre = P + wrel;
  double best = wpre, run = wpre;
  int bj = -1;
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    if (j >= kJLo && j <= kJHi && (bj < 0 || fabs(run) > fabs(best)) && e0 + tid * kW + j < v.n) {
      best = run;
      bj = j;
    }
    const float e = xs(tid * kW + j);
    if (isfinite(e)) run += (double)e;
  }
  if (bj < 0) {  // (a last window shorter than kJLo + 1 elements)
    best = wpre;
    bj = 0;
  }
  if (b == 0) {  // the chain's first element (a stretch: its fp64 prefix, P)
    best = v.p0 ? P : 0.0;
    bj = 0;
  }
  sbs[tid] = tid * kW + bj;  // tile-relative start
  sA[tid] = best;
  if (tid == kFrontT - 1) {
    // the next tile's first block start (same rule), for this tile's last block
    double r2 = P + ttotal, b2 = r2;
    int j2 = -1;
    for (int j = 0; j < kW; ++j) {
      if (j >= kJLo && j <= kJHi && (j2 < 0 || fabs(r2) > fabs(b2)) && e0 + kTile + j < v.n) {
        b2 = r2;
        j2 = j;
      }
      const float e = xs(kTile + j);
      if (isfinite(e)) r2 += (double)e;
    }
    sbs[kFrontT] = kTile + (j2 < 0 ? 0 : j2);
  }
  __syncthreads();
  int* bsg = v.bs + (int64_t)c * (v.nb + 1);
  if (b < v.nb) bsg[b] = (int)(e0 + sbs[tid]);
  if (b == v.nb - 1) bsg[v.nb] = (int)v.n;
  // group starts: the block of largest |start value| among blocks [kJLo,
  // kJHi] of each 16-block window (others only when none of those exists;
  // out-of-range blocks never win)
  const int wj = tid & (kGW - 1);
  double key = b < v.nb ? (wj >= kJLo && wj <= kJHi ? fabs(sA[tid]) : -0.5) : -1.0;
  int kid = b < v.nb ? b : INT_MAX;
  // (the row's lexicographic max by DPP: order-free, the same winner)
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    double ok;
    int oi;
    switch (st) {  // (unrolled: constant controls)
      case 0: ok = dpp_d<kRowBfly[0]>(key); oi = dpp_i<kRowBfly[0]>(kid); break;
      case 1: ok = dpp_d<kRowBfly[1]>(key); oi = dpp_i<kRowBfly[1]>(kid); break;
      case 2: ok = dpp_d<kRowBfly[2]>(key); oi = dpp_i<kRowBfly[2]>(kid); break;
      default: ok = dpp_d<kRowBfly[3]>(key); oi = dpp_i<kRowBfly[3]>(kid); break;
    }
    if (ok > key || (ok == key && oi < kid)) {
      key = ok;
      kid = oi;
    }
  }
  const int q = b / kGW;
  if ((tid & (kGW - 1)) == 0 && q < v.ng) {
    int* gsg = v.gs + (int64_t)c * (v.ng + 1);
    gsg[q] = q == 0 ? 0 : kid;
    if (q == v.ng - 1) gsg[v.ng] = v.nb;
  }
  // superblock start: the group of largest |start| among the tile's groups
  if ((tid & (kGW - 1)) == 0) {
    gkey[tid / kGW] = q < v.ng ? key : -1.0;
    gid[tid / kGW] = q;
  }
  __syncthreads();
  if (tid == 0) {
    double bk = -2.0;
    int bq = 0;
    for (int i = 0; i < kKW; ++i) {
      const double k = i >= kJLo && i <= kJHi ? gkey[i] : (gkey[i] >= 0.0 ? -0.5 : -1.0);
      if (k > bk) {
        bk = k;
        bq = gid[i];
      }
    }
    int* ksg = v.ks + (int64_t)c * (v.nk + 1);
    ksg[t] = t == 0 ? 0 : bq;
    if (t == v.nk - 1) ksg[v.nk] = v.ng;
  }
  // the block's unmonitored float32 run from its fp64 guess
  double incv = 0.0;
  if (b < v.nb) {
    const int s0 = sbs[tid];
    const int s1 = b == v.nb - 1 ? (int)(v.n - e0) : sbs[tid + 1];
    const float G = b == 0 && !v.p0 ? 0.0f : (float)sA[tid];
    float s = G;
    double fsum = 0.0;
    for (int i = s0; i < s1; ++i) {
      const float e = xs(i);
      s = s + e;
      if (isfinite(e)) fsum += (double)e;
    }
    incv = isfinite(s) && isfinite(G) ? (double)s - (double)G : fsum;
    v.inc[(int64_t)c * v.nb + b] = incv;
  }
  double itot;
  const double ipv = block_scan_excl<kFrontT>(incv, lds, &itot);
  if (b < v.nb) v.ipre[(int64_t)c * v.nb + b] = ipv;
  if (tid == 0) v.tinc[(int64_t)c * v.nk + t] = itot;
}

// ---- 3: leaf, group and superblock maps, one workgroup per superblock -------------
// One workgroup per (superblock, chain) builds every map of the superblock:
//   leaves      one lane per block (<= 511 blocks: one round of 512 lanes) runs
//               candidate 0 -- the block's guess G -- through the block's
//               elements (staged in LDS).  When that run rounds on no grid
//               coarser than G's own (its lattice need <= e0: m = 0), the map
//               needs no other candidate: any start on G's grid is G + d, d a
//               multiple of every step's grid, and the run's window says which
//               d keep every step's rounding.  That is ~99.7% of an ICP loop's
//               blocks (tools/seqsum_incr_sim.py's leaf histogram: m = 0
//               1,295,842 / m = 1 3,751 / m = 2 296 / exact-only 111 over 24
//               iterations at 640x480); the rest list their candidates 1..3 in
//               LDS and run them in one extra round, then m is the largest need
//               over the four runs as before.  (r05: four lanes per block,
//               every block, in a kernel of its own -- 5.3M VALU instructions
//               an iteration, three quarters of them for entries m = 0 drops.)
//   groups      lanes (group, candidate) listed compactly: every group's
//               candidate 0, then the candidates 1..R-1 of groups whose
//               lattice needs them (97.7% need none), composed through the
//               group's leaf maps from LDS;
//   superblock  lanes r < R (R = 1 for 87% of superblocks, 2 for 11%)
//               composed through the group maps.
// Every map is a valid statement about its own runs whatever the guess (a
// wrong guess only costs hits), so the walk's results never depend on this
// kernel's choices.  Leaf and group maps go to global memory for the walk's
// descents.
// k_sq_leaves: 320 threads (a lane per block; blocks past the first 320 of
// a superblock -- rare: ~256 on average -- take a second round), five
// workgroups per CU (25 waves, <= 7 per SIMD: <= 72 registers; LDS <= 32
// KB each; six, <= 64 registers, spilled 16 B).  k_sq_comp: one wavefront.  r20 before the split: one workgroup
// of 512 threads, three per CU, 38.1k it/s; of 320, five per CU, 40.8k.
constexpr int kBuildT = 320;
#ifndef RST_SQ_LEAVES_PER_CU
#define RST_SQ_LEAVES_PER_CU 5  // (r20b / r20j: 6 -> 5, 41.1k -> 41.3k it/s alone, part of r20j's combination)
#endif
constexpr int kLeavesPerCU = RST_SQ_LEAVES_PER_CU;
constexpr int kLeavesWaves = (kLeavesPerCU * kBuildT / kWave + 3) / 4;
static_assert(kBuildT >= kWave && kBuildT % kWave == 0, "leaf workgroup size");
// the single-stream k_sq_build (a pair alone: latency, not residency): a lane
// for every block of the largest superblock, one leaf round (r24: at 320
// threads, the superblocks past 320 blocks took a second round and set the
// kernel's time, 39 -> 45 us an iteration of a lone pair)
constexpr int kBuildT1 = 512;
static_assert(kBuildT1 >= kMaxSbBlocks, "one leaf round");
static_assert(sizeof(Leaf) == 64, "a leaf map is four int4");
constexpr int kListCap = (kLeafR - 1) * kMaxSbBlocks;
constexpr int16_t kNeedNone = INT16_MIN;  // kNoNeed in 16 bits
static_assert((kMaxSbBlocks << 2 | 3) <= 0xffff && (kMaxSbGroups << 4 | 15) <= 0xffff, "list codes in 16 bits");
static_assert(kListCap >= kMaxSbGroups * kGroupR, "the group list shares the leaf list's storage");

// A composite lane's step through a child map, without branches (the
// lanes of a wavefront take different cases in the same step; a chain of
// divergent branches cost ~1k clocks a step): comp_off the offset k of x in
// the child's grid (`ok` cleared when the child is unusable or x is off its
// grid), comp_apply the entry r = k mod 2^m -- the same arithmetic as
// `through` (rst_seqsum.hpp); once `ok` is false nothing changes.
__device__ __forceinline__ int comp_off(float x, const MapHdr& h, int mmax, bool& ok) {
  const bool hv = !(h.flags & kOpaque) && h.m >= 0 && h.m <= mmax;
  const uint32_t vb = __float_as_uint(x), gb = __float_as_uint(h.G);
  const bool same = ((vb ^ gb) >> 23) == 0;
  const int d = (int)(vb & 0x7fffffu) - (int)(gb & 0x7fffffu);
  int k = (gb >> 31) ? -d : d;
  bool kok = same;
  const bool slow = ok && hv && !same;
  if (__ballot(slow) != 0) {  // (rare: x in another binade than G)
    if (slow) {
      const OffK o = offset_units_slow(x, h.G, h.e0);
      k = o.k;
      kok = o.ok != 0;
    }
  }
  ok = ok && hv && kok;
  return k;
}
__device__ __forceinline__ void comp_apply(float& x, double& clo, double& chi, bool& ok, const MapHdr& h, int k,
                                           const MapEnt& en) {
  const int du = k - (k & ((1 << (ok ? h.m : 0)) - 1));
  const bool inwin = en.LOu <= du && du <= en.HIu;
  const float dd = ldexpf((float)du, h.e0);
  const float o = en.E + dd;
  const bool ebig = fabsf(en.E) >= fabsf(dd);
  const bool exact = ebig ? (o - en.E == dd) : (o - dd == en.E);
  ok = ok && inwin && (du == 0 || exact);
  clo = ok ? fmax(clo, ldexp((double)(en.LOu - du), h.e0)) : clo;
  chi = ok ? fmin(chi, ldexp((double)(en.HIu - du), h.e0)) : chi;
  x = ok ? (du == 0 ? en.E : o) : x;
}

__device__ __forceinline__ float cand(float G, int e0, int r) {
  return (float)((double)G + ldexp((double)r, e0));
}

// One speculative step in the integers (scalar ALU): the end E_r + du 2^e0
// as E_r's bits plus du in E_r's grid -- what the float formula gives
// whenever the step is valid (the offset rule keeps E_r + d in E_r's binade,
// d a multiple of its grid), up to a power-of-two E_r, which the lanes'
// checks (the float formula) catch like any unverified step.  sh = e0 minus
// E_r's grid exponent, per entry, computed lane-parallel beside the entries
// (step_shift).  r06: the float formula's VALU round trip (v_readfirstlane,
// cvt, ldexp, sub) made a step ~250 clocks.
__device__ __forceinline__ int step_shift(float E, int e0) {
  return e0 - (max((int)((__float_as_uint(E) >> 23) & 0xffu), 1) - 150);
}
__device__ __forceinline__ int step_bits(int Eb, int du, int sh) {
  // (shift counts masked to 5 bits as the scalar shifts take them: a clamp
  // selects v_med3 and moves the whole chain to vector registers; an
  // out-of-range shift only yields a value the checks reject)
  const int l = max(sh, 0) & 31, rr = max(-sh, 0) & 31;
  const int u = (du << l) >> rr;
  return Eb >= 0 ? Eb + u : Eb - u;  // (a negative float's bits are a negative int)
}

// The speculative chain of a run of maps as a parallel prefix (r06: a
// step-by-step scalar chain cost ~250 clocks a step, its dependent
// scalar / v_readlane round trips).  For a fixed residue r the step of
// lane q's map is affine in the input's bits x (same sign and binade as G,
// what the checks verify): x' = Eb + sE 2^sh (sG (x - gb) - r) =
// A_q + B_q x, B_q = sE sG 2^sh.  An inclusive scan of (A, B) over the
// chunk's lanes (DPP row shifts, lanes < 16: kWalkC) composes the steps;
// lane q's input is the composition of the steps before it applied to
// sb0.  A, B are dyadic rationals far inside double's 53 bits (x < 2^31,
// |sh| small), so the prefix is exact wherever the steps are valid; a value
// that is not an int32 becomes NaN bits, which no check accepts.
template <int CTRL>
__device__ __forceinline__ int dpp_row(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_row(double old, double x) {
  const uint2 o = __builtin_bit_cast(uint2, old), u = __builtin_bit_cast(uint2, x);
  const int lo = __builtin_amdgcn_update_dpp((int)o.x, (int)u.x, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)o.y, (int)u.y, CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, make_uint2((unsigned)lo, (unsigned)hi));
}
template <int D>
__device__ __forceinline__ void affine_scan_step(double& A, int& e, int& sg) {
  constexpr int kRowShr = 0x110 + D;  // DPP row_shr:D (lanes below D in their row keep `old`)
  const double Ap = dpp_row<kRowShr>(0.0, A);  // (identity: A = 0, B = +1)
  const int ep = dpp_row<kRowShr>(0, e);
  const int sp = dpp_row<kRowShr>(1, sg);
  A = A + (double)sg * ldexp(Ap, e);
  e += ep;
  sg *= sp;
}
// lane q (< nq <= 16): Eb, sh, gb, r of its map's step; returns lane q's
// input (lane 0: sb0), lane nq the chunk's end
__device__ __forceinline__ int affine_hist(int sb0, int Eb, int sh, int gb, int r, int nq) {
  const int lane = threadIdx.x & (kWave - 1);
  const bool on = lane < nq;
  const int sgG = (gb >> 31) | 1, sgE = (Eb >> 31) | 1;
  double A = on ? (double)Eb - (double)sgE * ldexp((double)((int64_t)sgG * gb + r), sh) : 0.0;
  int e = on ? sh : 0;
  int sg = on ? sgE * sgG : 1;
  affine_scan_step<1>(A, e, sg);
  affine_scan_step<2>(A, e, sg);
  affine_scan_step<4>(A, e, sg);
  affine_scan_step<8>(A, e, sg);
  const double val = A + (double)sg * ldexp((double)sb0, e);
  const bool okv = val == rint(val) && val >= -2147483648.0 && val < 2147483648.0;
  const int vi = okv ? (int)(int64_t)val : 0x7fc00000;
  const int h = __builtin_amdgcn_update_dpp(0, vi, 0x138, 0xf, 0xf, false);  // wave_shr:1: lane q <- q - 1 (no LDS trip)
  return lane == 0 ? sb0 : h;
}

// A chunk's speculative inputs from sb0 (lane q < nq: map maps[ql], ql = q):
// every step with residue 0 first; when a map of the chunk has several
// residues, again with each lane's residue from the first pass's input (right
// whenever the steps before it were)
template <class Map>
__device__ __forceinline__ int spec_hist(int sb0, const Map* maps, int ql, const MapHdr& hl, int gbl, int sgl,
                                         int mkl, int nq) {
  const int lane = threadIdx.x & (kWave - 1);
  float El = maps[ql].e[0].E;
  int hist = affine_hist(sb0, (int)__float_as_uint(El), step_shift(El, hl.e0), gbl, 0, nq);
  if (__ballot(lane < nq && mkl != 0) != 0) {
    const int rl = (((hist - gbl) ^ sgl) - sgl) & mkl;
    El = maps[ql].e[rl].E;
    hist = affine_hist(sb0, (int)__float_as_uint(El), step_shift(El, hl.e0), gbl, rl, nq);
  }
  return hist;
}


// One candidate x through maps[0, n) (LDS) -- the same statement as
// comp_off / comp_apply map after map, made by the whole wavefront: up to
// kChainC maps a round, the values speculated in scalar registers
// (step_bits, the entries by v_readlane), then every step checked on its
// own lane (same binade, usable header, in window, exact, the value the
// speculation carried on) and the window narrowed by a reduction over the
// verified lanes.  A step that fails its check -- x in another binade than
// the map's G, or a power-of-two end -- is taken by comp_off / comp_apply
// themselves, so the result is theirs, bit for bit.  False: the candidate
// cannot pass (no map for it).  r06: a lane stepping through the maps with
// an LDS read per step took ~13k clocks for a superblock's 16 groups.
constexpr int kChainC = 16;
// superblock candidates taken by comp_chain (more: a lane each); the group
// composites are a lane each (r07: by comp_chain 19.7k -> 17.5k clocks a
// group phase, the value unchanged)
constexpr int kSbChainR = 4;
template <class Map>
__device__ __forceinline__ bool comp_chain(float& x, double& clo, double& chi, const Map* maps, int n, int mmax) {
  const int lane = threadIdx.x & (kWave - 1);
  n = __builtin_amdgcn_readfirstlane(n);  // (every lane's alike: a scalar loop)
  int q0 = 0;
  while (q0 < n) {
    const int nq = __builtin_amdgcn_readfirstlane(min(n - q0, kChainC));
    const Map* mp = maps + q0;
    const int ql = min(lane, nq - 1);
    const MapHdr hl = mp[ql].h;
    const int gbl = (int)__float_as_uint(hl.G);
    const int sgl = gbl >> 31;
    const int mkl = (1 << min(hl.m & 7, mmax)) - 1;
    const int sb0 = __builtin_amdgcn_readfirstlane((int)__float_as_uint(x));
    int hist = spec_hist(sb0, mp, ql, hl, gbl, sgl, mkl, nq);
    const int nxb = __builtin_amdgcn_update_dpp(0, hist, 0x130, 0xf, 0xf, false);  // wave_shl:1: lane q <- q + 1
    bool okl;
    double lo, hi;
    {
      const bool same = (((uint32_t)hist ^ (uint32_t)gbl) >> 23) == 0u;
      const bool hv = !(hl.flags & kOpaque) && hl.m >= 0 && hl.m <= mmax;
      const int kk = ((hist - gbl) ^ sgl) - sgl;
      const int r = kk & mkl;
      const MapEnt en = mp[ql].e[r];
      const int du = kk - r;
      const bool inwin = en.LOu <= du && du <= en.HIu;
      const float dd = ldexpf((float)du, hl.e0);
      const float o = en.E + dd;
      const bool ebig = fabsf(en.E) >= fabsf(dd);
      const bool exact = ebig ? (o - en.E == dd) : (o - dd == en.E);
      const float xo = du == 0 ? en.E : o;
      okl = lane < nq && same && hv && inwin && (du == 0 || exact) && (int)__float_as_uint(xo) == nxb;
      lo = ldexp((double)(en.LOu - du), hl.e0);
      hi = ldexp((double)(en.HIu - du), hl.e0);
    }
    const uint64_t bad = __ballot(!okl) & ((1ull << nq) - 1);
    const int qf = bad ? (int)__builtin_ctzll(bad) : nq;
    // the verified steps' windows (lanes < qf < kChainC <= 16: one row)
    lo = lane < qf ? lo : -INFINITY;
    hi = lane < qf ? hi : INFINITY;
    static_assert(kChainC == 16, "one row");
    lo = fmax(lo, dpp_d<kRowBfly[0]>(lo));
    hi = fmin(hi, dpp_d<kRowBfly[0]>(hi));
    lo = fmax(lo, dpp_d<kRowBfly[1]>(lo));
    hi = fmin(hi, dpp_d<kRowBfly[1]>(hi));
    lo = fmax(lo, dpp_d<kRowBfly[2]>(lo));
    hi = fmin(hi, dpp_d<kRowBfly[2]>(hi));
    lo = fmax(lo, dpp_d<kRowBfly[3]>(lo));
    hi = fmin(hi, dpp_d<kRowBfly[3]>(hi));
    clo = fmax(clo, rd_lane0(lo));
    chi = fmin(chi, rd_lane0(hi));
    x = __int_as_float(__builtin_amdgcn_readlane(hist, qf));
    if (qf == nq) {
      q0 += nq;
      continue;
    }
    // step q0 + qf by the lane statement itself (every lane alike)
    const MapHdr H = mp[qf].h;
    bool ok = true;
    const int kq = comp_off(x, H, mmax, ok);
    if (!ok) return false;
    comp_apply(x, clo, chi, ok, H, kq, mp[qf].e[kq & ((1 << H.m) - 1)]);
    if (!ok) return false;
    q0 += qf + 1;
  }
  return true;
}

// the wavefront's largest v, v in [lo, lo + 2^B): B ballots, most significant
// bit first -- no cross-lane data move (a shuffle butterfly is six LDS-unit
// round trips, ~600 clocks)
template <int B>
__device__ __forceinline__ int wave_max_small(int v, int lo = 0) {
  const int u = v - lo;
  int hi = 0;
#pragma unroll
  for (int b = B - 1; b >= 0; --b) {
    const int t = hi | (1 << b);
    hi = __ballot(u >= t) != 0 ? t : hi;
  }
  return hi + lo;
}

// A leaf map in LDS: its header and entry 0 (the only entry of ~99.7% of
// the leaves, m = 0); entries 1..3 of the others are read from the global
// map (written before the group phase) by the rare composite step that
// needs them.  aux: during the leaf phase, candidate 0's lattice need.
struct LeafL {  // 8 dwords: two int4
  MapHdr h;
  MapEnt e0;
  int aux;
};
static_assert(sizeof(LeafL) == 32, "an LDS leaf map is two int4");
// a group map in LDS: the global GroupMap without its padding, xo = the
// exact-only flag (the global map's pad[0])
struct GroupMapL {
  MapHdr h;
  MapEnt e[kGroupR];
  int xo;
};
constexpr int kGroupMapLW = (int)(sizeof(GroupMapL) / 4);
static_assert(kGroupMapLW == 53 && offsetof(GroupMap, pad) == 4 * 52, "GroupMapL = GroupMap's first 53 dwords");

// The maps are built by two kernels per superblock (r20): k_sq_leaves (320
// threads, a lane per block: the leaf runs) and k_sq_comp (one wavefront:
// the group and superblock composites, the leaf maps read back from global
// memory).  Until r20 one workgroup did both, and most of its time -- the
// composites, one or two wavefronts' dependent chains -- held the LDS and
// the wave slots its leaf phase needed: three workgroups per CU, 49 KB of
// LDS each (r06: 76 KB and two per CU with the elements staged).
struct LeafLds {  // ~24.5 KB: six workgroups per CU
  LeafL lf[kMaxSbBlocks];
  int sbs[kMaxSbBlocks + 1];   // block starts, relative to the superblock's first element
  int16_t xneed[kMaxSbBlocks][kLeafR - 1];  // the extra candidates' lattice needs (kNeedNone: none)
  // extra leaf candidates (block << 2 | r): up to kLeafR - 1 per block (a
  // stream of exact ties needs them for most blocks)
  uint16_t list[kListCap];
  int nlist;
  double base[2];              // fp64 increments of the tiles before the superblock's first
                               // tile and before the next
};
struct CompLds {  // ~7.7 KB
  GroupMapL gm[kMaxSbGroups];
  int sgs[kMaxSbGroups + 1];   // group starts, relative to its first block
  uint16_t list[kMaxSbGroups * kGroupR];  // (group << 4 | r): every group's candidate 0 first
  int nlist;
  int bad;
};
static_assert(sizeof(LeafLds) + sizeof(CompLds) <= 160 * 1024 / kLeavesPerCU, "the map workgroups' LDS per CU");

// one monitored run of a block from candidate r: its len <= 2 kW - 1
// elements X[a], X[a + 1], ... (the chain's SoA row, rows padded to 64
// floats) into registers first -- nine 16-byte loads from a's 16-byte
// boundary, clamped inside the row -- so the run's chain waits on no load;
// register j is step j - a mod 4 (steps predicated per lane: a select by the
// lane's offset became an indexed scratch access); at most `wmax` + 3 steps
// (the wavefront's longest block, uniform)
__device__ __forceinline__ void leaf_run(Run& p, const float* __restrict__ X, int64_t ns, int64_t a, int len,
                                         int wmax, float G, int e0, int r) {
  constexpr int kL4 = (2 * kW - 1 + 3 + 3) / 4;  // float4 loads covering a mod 4 + len
  run_init(p, cand(G, e0, r));
  const int64_t a4 = a >> 2, last4 = (ns >> 2) - 1;
#if defined(__HIP_DEVICE_COMPILE__)
  const auto* X4 = (const __attribute__((address_space(1))) float4*)X;  // (global loads, not flat)
#else
  const float4* X4 = reinterpret_cast<const float4*>(X);
#endif
  float w[4 * kL4];
#pragma unroll
  for (int j = 0; j < kL4; ++j) {
    const float4 t = X4[min(a4 + j, last4)];
    w[4 * j] = t.x;
    w[4 * j + 1] = t.y;
    w[4 * j + 2] = t.z;
    w[4 * j + 3] = t.w;
  }
  const int off = (int)(a & 3);
  // (unrolled and predicated, not a break: w[j] stays a register)
#pragma unroll
  for (int j = 0; j < 2 * kW - 1 + 3; ++j) {
    if (j < wmax + 3) {
      if (j >= off && j < off + len) run_step(p, w[j], e0);
    }
  }
}

__device__ __forceinline__ MapEnt leaf_ent(const Run& p, int e0) {
  MapEnt en;
  en.E = p.s;
  en.LOu = lo_units((double)p.lo, e0);
  en.HIu = hi_units((double)p.hi, e0);
  if (p.opaque) {
    en.LOu = 1;
    en.HIu = 0;
  }
  return en;
}

// LDS ordering within a one-wavefront workgroup (no s_barrier: the fused
// kernel's other wavefronts have ended)
__device__ __forceinline__ void sq_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// the superblock's group / block / element ranges, checked before each
// dependent load (a bad table stops the workgroup instead of reading out of
// range); false: stop
struct SbRange {
  int ga, gb, ba, bb, ea, eb;
};
__device__ __forceinline__ bool sb_range(const SqView& v, int k, int c, bool flag, SbRange& r) {
  const int* bsg = v.bs + (int64_t)c * (v.nb + 1);
  const int* gsg = v.gs + (int64_t)c * (v.ng + 1);
  const int* ksg = v.ks + (int64_t)c * (v.nk + 1);
  r.ga = ksg[k];
  r.gb = ksg[k + 1];
  if (r.ga < 0 || r.gb > v.ng || r.gb - r.ga < 1 || r.gb - r.ga > kMaxSbGroups) {
    if (flag) atomicOr(v.err, 1);
    return false;
  }
  r.ba = gsg[r.ga];
  r.bb = gsg[r.gb];
  if (r.ba < 0 || r.bb > v.nb || r.bb - r.ba < 1 || r.bb - r.ba > kMaxSbBlocks) {
    if (flag) atomicOr(v.err, 1);
    return false;
  }
  r.ea = bsg[r.ba];
  r.eb = bsg[r.bb];
  if (r.ea < 0 || r.eb > v.n || r.eb - r.ea < 1 || r.eb - r.ea > kMaxSbElems) {
    if (flag) atomicOr(v.err, 1);
    return false;
  }
  return true;
}

// k_sq_leaves: every leaf map of superblock k of chain c (global v.leaf)
// (lds_maps: the maps' headers and entries 0 also left in W.lf, the fused
// kernel's composites read them there)
// (T threads: k_sq_leaves_b T, the single-stream k_sq_build T1)
template <int T>
__device__ __forceinline__ void sq_leaf_body(const SqView& v, const int k, const int c, LeafLds& W,
                                             bool lds_maps) {
  RST_TL(v.tl, v.it, 4);
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  long long* clk = v.clk + ((int64_t)c * v.nk + k) * 8;
  if (tid == 0) clk[0] = (long long)__builtin_amdgcn_s_memtime();
  SbRange sr;
  if (!sb_range(v, k, c, tid == 0, sr)) return;
  const int ba = sr.ba, ea = sr.ea;
  const int nblk = sr.bb - sr.ba, nel = sr.eb - sr.ea;
  const int* bsg = v.bs + (int64_t)c * (v.nb + 1);
  const float* X = v.soa + (int64_t)c * v.ns;
  const double* ipre = v.ipre + (int64_t)c * v.nb;
  Leaf* leafg = v.leaf + (int64_t)c * v.nb + ba;  // the superblock's leaf maps (global)
  // (every staging load issued before the first store -- r22: the block
  // starts and the tiles' increments were two dependent trips more; the
  // first round's increment prefixes stay in flight across the barrier)
  const double iv0 = tid < nblk ? ipre[ba + tid] : 0.0;
  constexpr int kSbR = (kMaxSbBlocks + 1 + T - 1) / T;  // block starts per thread
  int sb[kSbR];
#pragma unroll
  for (int r = 0; r < kSbR; ++r) {
    const int i = tid + r * T;
    sb[r] = i <= nblk ? bsg[ba + i] : 0;
  }
  const double* ti = v.tinc + (int64_t)c * v.nk;
  constexpr int kTiR = 4;  // the tiles' increments per lane in flight
  double tv[kTiR];
  double s = 0.0;
  if (tid < kWave) {
#pragma unroll
    for (int r = 0; r < kTiR; ++r) tv[r] = lane + r * kWave < k ? ti[lane + r * kWave] : 0.0;
    for (int i = lane + kTiR * kWave; i < k; i += kWave) s += ti[i];  // (> 256 tiles: a 1M-element chain)
  }
  const double tk = tid == kWave - 1 && k < v.nk ? ti[k] : 0.0;
#pragma unroll
  for (int r = 0; r < kSbR; ++r) {
    const int i = tid + r * T;
    if (i <= nblk) W.sbs[i] = sb[r] - ea;
  }
  if (tid == 0) W.nlist = 0;
  if (tid < kWave) {  // the tiles' increments before tile k
#pragma unroll
    for (int r = 0; r < kTiR; ++r) s += tv[r];
    s = wave_sum_last(s);  // (a guess's offset: any association)
    if (lane == kWave - 1) {
      const double q = v.p0 ? v.p0[c] : 0.0;  // (a stretch of a longer chain)
      W.base[0] = s + q;
      W.base[1] = s + q + tk;
    }
  }
  __syncthreads();
  if (tid == 0) clk[1] = (long long)__builtin_amdgcn_s_memtime();
  // -- candidate 0 per block, a lane each (rounds of T blocks): its
  // header, entry and lattice need to LDS, h.m = 1 marking a block whose
  // other candidates are listed
  for (int b0 = 0; b0 < nblk; b0 += T) {
    const int bi = b0 + tid;
    const bool act = bi < nblk;
    const int b = ba + bi;
    float G = 0.0f;
    int e0 = -149, a0 = 0, len = 0;
    if (act) {
      const double iv = b0 == 0 ? iv0 : ipre[b];
      a0 = W.sbs[bi];
      len = W.sbs[bi + 1] - a0;
      if (a0 < 0 || len < 1 || len > 2 * kW - 1 || a0 + len > nel) {
        atomicOr(v.err, 32);
        a0 = len = 0;
      }
      // a superblock's blocks lie in tile k and tile k + 1
      const double base = (b / kBlocksPerTile) == k ? W.base[0] : W.base[1];
      G = candidate_base(b == 0 && !v.p0 ? 0.0f : (float)(base + iv), kLeafR);
      e0 = grid_exp(G);
    }
    // the wavefront's longest block bounds the unrolled steps
    const int wmax = wave_max_small<5>(len);  // (a block <= 2 kW - 1 elements)
    Run p;
    if (wmax > 0) {
      leaf_run(p, X, v.ns, (int64_t)ea + a0, len, wmax, G, e0, 0);
    } else {
      run_init(p, 0.0f);
    }
    if (act && len == 0) p.opaque = true;  // (a bad block: no map)
    const int m0 = p.need == kNoNeed ? 0 : max(0, p.need - e0);
    const bool more = act && !p.opaque && m0 >= 1 && m0 <= kLeafM;
    if (more) {
      const int at = atomicAdd(&W.nlist, kLeafR - 1);
      if (at + kLeafR - 1 <= kListCap) {  // (always: kListCap covers every block)
#pragma unroll
        for (int r = 1; r < kLeafR; ++r) W.list[at + r - 1] = (uint16_t)(bi << 2 | r);
      } else {
        atomicOr(v.err, 64);
      }
    }
    if (act) W.lf[bi] = LeafL{MapHdr{G, e0, more ? 1 : 0, p.opaque ? kOpaque : 0}, leaf_ent(p, e0), p.need};
  }
  __syncthreads();
  {
    // the listed extra candidates, one lane each (rare; uniform skip): their
    // entries straight to the global map, their needs to LDS
    const int nl = min(W.nlist, kListCap);
    for (int j0 = 0; j0 < nl; j0 += T) {
      const int j = j0 + tid;
      const int code = j < nl ? W.list[j] : 0;
      const int bl = min(code >> 2, nblk - 1), r = code & 3;
      const int xa = j < nl ? W.sbs[bl] : 0, xl = j < nl ? W.sbs[bl + 1] - xa : 0;
      const float xG = j < nl ? W.lf[bl].h.G : 0.0f;
      const int xe0 = grid_exp(xG);
      const int wmax = wave_max_small<5>(xl);
      if (wmax > 0) {
        Run q;
        leaf_run(q, X, v.ns, (int64_t)ea + xa, xl, wmax, xG, xe0, r);
        if (j < nl) {
          leafg[bl].e[r] = leaf_ent(q, xe0);
          W.xneed[bl][r - 1] = q.need == kNeedNone ? kNeedNone : (int16_t)max(-32767, min(32767, q.need));
        }
      }
    }
  }
  __syncthreads();
  // the leaf maps: lattice need over the candidates -> m, the map whole to
  // global memory
  for (int bi = tid; bi < nblk; bi += T) {
    const LeafL L = W.lf[bi];
    const bool more = L.h.m != 0;
    int need = L.aux;
    if (more)
#pragma unroll
      for (int r = 1; r < kLeafR; ++r) {
        const int xn = W.xneed[bi][r - 1];
        need = max(need, xn == kNeedNone ? kNoNeed : xn);
      }
    const int e0 = L.h.e0;
    const int mneed = need == kNoNeed ? 0 : max(0, need - e0);
    const bool exact_only = mneed > kLeafM;
    const int m = exact_only ? 0 : mneed;
    Leaf o;
    o.h = MapHdr{L.h.G, e0, m, L.h.flags};
    o.e[0] = L.e0;
#pragma unroll
    for (int r = 1; r < kLeafR; ++r) o.e[r] = more ? leafg[bi].e[r] : MapEnt{0.0f, 1, 0};
#pragma unroll
    for (int r = 0; r < kLeafR; ++r) {
      if (r >= (1 << m)) {
        o.e[r].LOu = 1;
        o.e[r].HIu = 0;
      } else if (exact_only) {
        o.e[r].LOu = max(o.e[r].LOu, 0);
        o.e[r].HIu = min(o.e[r].HIu, 0);
      }
    }
    leafg[bi] = o;
    if (lds_maps) W.lf[bi] = LeafL{o.h, o.e[0], 0};
  }
  if (tid == 0) clk[6] = (long long)__builtin_amdgcn_s_memtime();
}

// k_sq_comp (one wavefront): superblock k's group maps (v.grp) and its map
// (v.sbm), composed through the leaf maps k_sq_leaves left in global memory
// (the single-stream k_sq_build: through its LDS copy).  (r21a: staging the
// headers and entries 0 in LDS first measured no faster, 41.7k vs 41.6k)
__device__ __forceinline__ void sq_comp_body(const SqView& v, const int k, const int c, CompLds& W,
                                             const LeafL* lds_leaves) {
  const int lane = threadIdx.x & (kWave - 1);
  long long* clk = v.clk + ((int64_t)c * v.nk + k) * 8;
  if (lane == 0) clk[2] = (long long)__builtin_amdgcn_s_memtime();
  SbRange sr;
  if (!sb_range(v, k, c, false, sr)) return;  // (k_sq_leaves flagged it)
  const int ga = sr.ga, gb = sr.gb, ba = sr.ba;
  const int ngr = gb - ga, nblk = sr.bb - sr.ba;
  const int* gsg = v.gs + (int64_t)c * (v.ng + 1);
  const Leaf* leafg = v.leaf + (int64_t)c * v.nb + ba;
  // leaf i: lq[lqs i] its header, lq[lqs i + 1] entry 0 (the global map:
  // lqs = 4, and entry 1's E; the fused kernel's LDS copy: lqs = 2)
  const int4* lq = lds_leaves ? reinterpret_cast<const int4*>(lds_leaves) : reinterpret_cast<const int4*>(leafg);
  const int lqs = lds_leaves ? 2 : 4;
  if (lane <= ngr) W.sgs[lane] = gsg[ga + lane] - ba;
  if (lane == 0) {
    W.nlist = ngr;
    W.bad = 0;
  }
  sq_wave_sync();
  // -- groups: the lattice (lane per group), then lanes (group, candidate)
  if (lane < ngr) {
    const int gi = lane;
    const int c0 = W.sgs[gi], c1 = W.sgs[gi + 1];
    const bool gok = c0 >= 0 && c1 > c0 && c1 <= nblk && c1 - c0 <= 2 * kGW - 1;
    GroupMapL& o = W.gm[gi];
    int R = 1;
    if (!gok) {
      atomicOr(v.err, 2);
      W.bad = 1;
      o.h = MapHdr{0.0f, 0, 0, kOpaque};
      o.xo = 0;
    } else {
      const int4 h0 = lq[lqs * c0];
      int lat = h0.y + h0.z;
      // (unrolled and predicated: every header read in flight at once --
      // a rolled loop waited on each)
#pragma unroll
      for (int j = 1; j < 2 * kGW - 1; ++j) {
        if (c0 + j < c1) {
          const int4 hj = lq[lqs * (c0 + j)];  // (one read, no branch)
          lat = (hj.w & kOpaque) ? lat : max(lat, hj.y + hj.z);
        }
      }
      int m = max(0, lat - h0.y);
      const bool exact_only = m > kGroupM;  // (the windows clamped to 0 below)
      if (exact_only) m = 0;
      R = 1 << m;
      const float Gg = candidate_base(__int_as_float(h0.x), R);
      o.h = MapHdr{Gg, grid_exp(Gg), m, 0};
      o.xo = exact_only ? 1 : 0;
    }
    for (int r = 0; r < kGroupR; ++r) o.e[r] = MapEnt{0.0f, 1, 0};
    if (R > 1) {
      const int at = atomicAdd(&W.nlist, R - 1);
      for (int r = 1; r < R; ++r)
        if (at + r - 1 < kMaxSbGroups * kGroupR) W.list[at + r - 1] = (uint16_t)(gi << 4 | r);  // (always)
    }
  }
  sq_wave_sync();
  {
    const int nl = min(W.nlist, kMaxSbGroups * kGroupR);
    for (int j0 = 0; j0 < nl; j0 += kWave) {
      const int j = j0 + lane;
      const bool ea_ = j < nl;
      const int code = !ea_ ? 0 : (j < ngr ? j << 4 : W.list[j]);
      const int gi = code >> 4, r = code & (kGroupR - 1);
      const int c0 = W.sgs[gi], c1 = W.sgs[gi + 1];
      const bool gok = ea_ && c0 >= 0 && c1 > c0 && c1 <= nblk && c1 - c0 <= 2 * kGW - 1;
      const MapHdr gh = W.gm[gi].h;
      const bool exact_only = W.gm[gi].xo != 0;  // (a lattice beyond kGroupM)
      float x = cand(gh.G, gh.e0, r);
      double clo = -INFINITY, chi = INFINITY;
      bool ok = gok && !(gh.flags & kOpaque);
      // (leaves j + 1 and j + 2 -- header and entry 0 -- in flight while
      // leaf j is applied; entries 1..3 -- leaves with m >= 1 -- from the
      // global map by a uniform branch taken when a lane needs one)
      const int cc0 = gok ? c0 : 0, cc1 = gok ? c1 : 1;
      int4 q0 = lq[lqs * cc0], q1 = lq[lqs * cc0 + 1];
      const int j1 = lqs * min(cc0 + 1, cc1 - 1);
      int4 n0 = lq[j1], n1 = lq[j1 + 1];
      const int nst = wave_max_small<5>(cc1 - cc0);  // (a group <= 2 kGW - 1 blocks)
      for (int s = 0; s < nst; ++s) {
        const int jl = cc0 + s;
        const int j2 = lqs * min(jl + 2, cc1 - 1);
        const int4 p0 = lq[j2], p1 = lq[j2 + 1];
        const MapHdr h{__int_as_float(q0.x), q0.y, q0.z, q0.w};
        bool okj = ok && jl < cc1;
        const int kq = comp_off(x, h, kLeafM, okj);
        const int rr = kq & ((1 << (okj ? h.m : 0)) - 1);  // (m <= kLeafM when ok)
        MapEnt en{__int_as_float(q1.x), q1.y, q1.z};
        if (__ballot(rr != 0) != 0) {
          if (rr != 0) en = leafg[jl].e[rr];
        }
        comp_apply(x, clo, chi, okj, h, kq, en);
        ok = jl < cc1 ? okj : ok;
        q0 = n0;
        q1 = n1;
        n0 = p0;
        n1 = p1;
      }
      if (ea_ && ok) {
        if (exact_only) {
          clo = fmax(clo, 0.0);
          chi = fmin(chi, 0.0);
        }
        W.gm[gi].e[r] = MapEnt{x, lo_units(clo, gh.e0), hi_units(chi, gh.e0)};
      }
    }
  }
  sq_wave_sync();
  if (lane == 0) clk[3] = (long long)__builtin_amdgcn_s_memtime();
  GroupMap* grpg = v.grp + (int64_t)c * v.ng + ga;
  for (int i = lane; i < ngr * kGroupMapLW; i += kWave) {
    const int g = i / kGroupMapLW, w = i - g * kGroupMapLW;
    reinterpret_cast<int*>(grpg + g)[w] = reinterpret_cast<const int*>(W.gm + g)[w];
  }
  if (lane == 0) clk[4] = (long long)__builtin_amdgcn_s_memtime();
  // -- the superblock: lanes = candidates, up to 64
  SbMap* so = v.sbm + (int64_t)c * v.nk + k;
  if (lane == 0) {
    so->ga = ga;
    so->gb = gb;
    so->ba = ba;
    so->bb = sr.bb;
    so->ea = sr.ea;
    so->eb = sr.eb;
  }
  if (W.bad) {
    if (lane == 0) so->h.flags = kOpaque;
    return;
  }
  const int r = lane;
  const MapHdr h0 = W.gm[0].h;
  // the lattice: the groups' e0 + m, lane per group, max over the wavefront
  // (e0 + m in [-149, 105 + kGroupM]: 9 bits above -160)
  const int lat = wave_max_small<9>(lane < ngr ? W.gm[lane].h.e0 + W.gm[lane].h.m : h0.e0 + h0.m, -160);
  int m = max(0, lat - h0.e0);
  const bool exact_only = m > kSbM;
  if (exact_only) m = 0;
  const int R = 1 << m;
  const float Gs = candidate_base(h0.G, R);
  const int se0 = grid_exp(Gs);
  if (r == 0) so->h = MapHdr{Gs, se0, m, 0};
  MapEnt en{0.0f, 1, 0};
  if (R <= kSbChainR) {
    // few candidates (R = 1 for ~87% of superblocks): one after another,
    // each by the whole wavefront (comp_chain)
    for (int rc = 0; rc < R; ++rc) {
      float x = cand(Gs, se0, rc);
      double clo = -INFINITY, chi = INFINITY;
      if (comp_chain<GroupMapL>(x, clo, chi, W.gm, ngr, kGroupM)) {
        if (exact_only) {
          clo = fmax(clo, 0.0);
          chi = fmin(chi, 0.0);
        }
        if (r == rc) en = MapEnt{x, lo_units(clo, se0), hi_units(chi, se0)};
      }
    }
  } else if (r < R) {
    float x = cand(Gs, se0, r);
    double clo = -INFINITY, chi = INFINITY;
    bool ok = true;
    // (group j + 1's header in flight while group j is applied)
    MapHdr H = W.gm[0].h;
    for (int j = 0; j < ngr; ++j) {
      const MapHdr Hn = W.gm[min(j + 1, ngr - 1)].h;
      const int kq = comp_off(x, H, kGroupM, ok);
      comp_apply(x, clo, chi, ok, H, kq, W.gm[j].e[kq & ((1 << (ok ? H.m : 0)) - 1)]);
      H = Hn;
    }
    if (ok) {
      if (exact_only) {
        clo = fmax(clo, 0.0);
        chi = fmin(chi, 0.0);
      }
      en = MapEnt{x, lo_units(clo, se0), hi_units(chi, se0)};
    }
  }
  so->e[r] = en;
  if (lane == 0) clk[5] = (long long)__builtin_amdgcn_s_memtime();
}


// ---- 4: the walk -------------------------------------------------------------------
// One wavefront per chain.  The superblock maps of a chunk of kWalkC
// superblocks sit in registers -- lane r holds every superblock's entry r,
// lane q < kWalkC superblock q's header -- so a step is a few scalar
// reads (v_readlane) and integer / float ops on the exact running sum; the
// next chunk's loads are in flight meanwhile.  A failed check descends
// (from global memory) to the superblock's group maps, then a group's
// leaf maps, then a block's own float adds.
constexpr int kWalkC = 16;

struct WalkStats {
  int sb, sbh, g, gh, l, lh, ser;
};

// A descent loads its superblock's group maps and block starts in one trip;
// a group its maps miss loads that group's leaf maps and elements in a
// second (r06: the whole superblock at once, ~72 KB through one wavefront,
// took 8.5k clocks before the first group was tried).
constexpr int kGrpElems = (2 * kGW - 1) * (2 * kW - 1);  // a group's elements, bound
// A group its map misses: its leaf maps, or with RST_SQ_GROUP_SERIAL the
// reference's own adds over the whole group -- measured slower (r07b, bench
// pair 14's x chain over an align: 60.8M walker clocks vs 50.8M; the adds
// ran ~53 clocks an element inside the walk, k_sq_serial's 12 not reached).
#ifndef RST_SQ_GROUP_SERIAL
#define RST_SQ_GROUP_SERIAL 0
#endif

// s <- the reference's adds over xl[0, cnt) (LDS), in order: 32 elements a
// round read by every lane at the same addresses (broadcast) into 32
// registers, then 32 dependent v_add_f32 -- no cross-lane move in the chain
// (r07a: a v_readlane per element cost ~78 clocks an element).  Past cnt
// the round adds +0, which changes no bit: s, a chain value from +0, is
// never -0 (k_sq_serial's argument).
__device__ __forceinline__ void serial_adds(float& s, const float* xl, int cnt) {
  constexpr int kR = 32;
  cnt = __builtin_amdgcn_readfirstlane(cnt);
  for (int c0 = 0; c0 < cnt; c0 += kR) {
    float xr[kR];
#pragma unroll
    for (int i = 0; i < kR; ++i) xr[i] = c0 + i < cnt ? xl[c0 + i] : 0.0f;
#pragma unroll
    for (int i = 0; i < kR; ++i) s = s + xr[i];
  }
}

struct WalkLds {
  GroupMap g[kMaxSbGroups];      // the descent's superblock: its group maps,
  int gs[kWave];                 // group starts,
  int bs[kMaxSbBlocks + 1 + 63]; // block starts;
  Leaf l[2 * kGW - 1];           // the missed group's leaf maps
  float x[kGrpElems + 8];        // and elements (from a 16-byte boundary)
  WalkStats ws;   // the descent's counters (LDS: no stack slot in the walk)
  long long tclk[8];  // (statistics) the first descent's phase clocks
  long long tph[6];   // (statistics) every descent's clocks by phase: group load, group steps,
                      // leaf load, leaf steps, own adds, whole descents
  int tph_on;
  int64_t pos_nf;  // element index where s became non-finite, else -1
};

// map (header h, entries e[] by residue) applied to the exact s (all lanes agree)
__device__ __forceinline__ bool walk_try(float& s, const MapHdr& h, const MapEnt* e, int mmax) {
  if ((h.flags & kOpaque) || h.m < 0 || h.m > mmax) return false;
  int k;
  if (!offset_units(s, h, k)) return false;
  const int r = k & ((1 << h.m) - 1);
  float out;
  if (!apply_ent(k - r, h.e0, e[r], out)) return false;
  s = out;
  return true;
}

// superblock k by its group maps, leaf maps and own adds; pos_nf >= 0 when
// the sum became inf / NaN (the element after the block that made it so)
// (not inlined: the walk's unrolled fast path stays a few hundred
// instructions; an inlined copy per step thrashed the instruction cache)
// (the chain's tables as plain arguments: a reference to the kernel's view
// would copy the view to a stack slot, and every walk would start with
// scratch traffic)
struct DescArgs {
  const GroupMap* grp;
  const Leaf* leaf;
  const int* bsg;
  const int* gsg;
  const float* X;
  int* err;
  int64_t n;
  int nb, ng;
};

// Steps over maps[0, nq) (in LDS; at most kWalkC per call) from s,
// speculatively -- every step's input at once, the steps composed as a
// parallel prefix (spec_hist) -- then the checks lane-parallel, step q on
// lane q (s before step q is lane q of `hist`).  Returns the number of
// leading verified steps, s after them.
template <class Map>
__device__ __forceinline__ int spec_chunk(float& s, const Map* maps, int nq, int mmax) {
  const int lane = threadIdx.x;
  const int ql = min(lane, nq - 1);
  const MapHdr hl = maps[ql].h;
  const int gbl = (int)__float_as_uint(hl.G);
  const int sgl = gbl >> 31;
  const int mkl = (1 << min(hl.m & 7, mmax)) - 1;  // (clamped: r stays inside the entries)
  const int hist = spec_hist(__builtin_amdgcn_readfirstlane((int)__float_as_uint(s)), maps, ql, hl, gbl, sgl, mkl, nq);
  const int nxb = __builtin_amdgcn_update_dpp(0, hist, 0x130, 0xf, 0xf, false);  // wave_shl:1: lane q <- q + 1
  int okl;
  {
    const int kk = ((hist - gbl) ^ sgl) - sgl;
    const int r = kk & mkl;
    const MapEnt en = maps[ql].e[r];
    const int du = kk - r;
    const float a = en.E, b = -ldexpf((float)(r - kk), hl.e0);
    const float o = en.E - ldexpf((float)(r - kk), hl.e0);
    const bool abig = fabsf(a) >= fabsf(b);
    const float big = abig ? a : b, sml = abig ? b : a;
    okl = (lane < nq) & ((((uint32_t)hist ^ (uint32_t)gbl) >> 23) == 0u) & ((hl.flags & kOpaque) == 0) &
          ((unsigned)hl.m <= (unsigned)mmax) & (en.LOu <= du) & (du <= en.HIu) & ((o - big) == sml) &
          ((int)__float_as_uint(o) == nxb);
  }
  const uint64_t bad = __ballot(!okl) & ((1ull << nq) - 1);
  const int qf = bad ? (int)__builtin_ctzll(bad) : nq;
  s = __int_as_float(__builtin_amdgcn_readlane(hist, qf));
  return qf;
}
template <class Map>
__device__ __forceinline__ int spec_walk(float& s, const Map* maps, int nq, int mmax) {
  nq = __builtin_amdgcn_readfirstlane(min(nq, kWalkC));  // (uniform: a scalar loop)
  int done = 0;
  while (done < nq) {
    done += spec_chunk(s, maps + done, nq - done, mmax);
    if (done >= nq) break;
    // the step the speculation could not verify -- often only a residue the
    // prefix took from a wrong input, or s in another binade than G -- by the
    // map itself; a true miss ends the run
    if (!walk_try(s, maps[done].h, maps[done].e, mmax)) break;
    ++done;
  }
  return done;
}

// n pieces of kSz bytes from src (global) to dst (LDS) by LDS-DMA: no
// registers staged, every piece in flight at once (the caller waits)
#define RST_GLDS_COPY(NAME, SZ)                                                                            \
  __device__ __forceinline__ void NAME(void* dst, const void* src, int n) {                               \
    const int lane = threadIdx.x;                                                                         \
    const char* sp = static_cast<const char*>(src);                                                       \
    char* dp = static_cast<char*>(dst);                                                                   \
    for (int j = 0; j * kWave < n; ++j) {                                                                 \
      const int i = j * kWave + lane;                                                                     \
      if (i < n)                                                                                          \
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(sp + (size_t)i * SZ), \
                                         (__attribute__((address_space(3))) void*)(dp + (size_t)j * kWave * SZ), \
                                         SZ, 0, 0);                                                       \
    }                                                                                                     \
  }
RST_GLDS_COPY(glds_copy16, 16)
RST_GLDS_COPY(glds_copy4, 4)
#undef RST_GLDS_COPY

// a value every lane holds alike, made scalar: a non-inlined function's
// arguments arrive in vector registers, and the compiler then treats every
// branch and loop on them as divergent (r06: exec-mask loops throughout
// the descent)
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni64(int64_t x) {
  const uint64_t u = (uint64_t)x;
  return (int64_t)(((uint64_t)(uint32_t)uni((int)(u >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)u));
}
template <class T>
__device__ __forceinline__ T* uni_ptr(T* p) {
  return reinterpret_cast<T*>(uni64(reinterpret_cast<int64_t>(p)));
}

__device__ __noinline__ float walk_descend(const DescArgs va, const int ga_, const int gb_, const int ba_,
                                           const int bb_, const int ea_, const int eb_, float s, WalkLds& W) {
  const DescArgs v{uni_ptr(va.grp), uni_ptr(va.leaf), uni_ptr(va.bsg), uni_ptr(va.gsg), uni_ptr(va.X),
                   uni_ptr(va.err), uni64(va.n), uni(va.nb), uni(va.ng)};
  const int ga = uni(ga_), gb = uni(gb_), ba = uni(ba_), bb = uni(bb_), ea = uni(ea_), eb = uni(eb_);
  int64_t& pos_nf = W.pos_nf;
  WalkStats& ws = W.ws;
  const int lane = threadIdx.x;
  const bool stamp = ws.g == 0 && lane == 0;  // (the first descent's phases)
  if (stamp) W.tclk[0] = (long long)__builtin_amdgcn_s_memtime();
  const bool ph = uni(W.tph_on) != 0;
  long long tp0 = ph ? (long long)__builtin_amdgcn_s_memtime() : 0, tpl = tp0;
  auto phase = [&](int j) {  // (statistics: the clocks since the last mark to phase j)
    if (ph) {
      const long long t = (long long)__builtin_amdgcn_s_memtime();
      if (lane == 0) W.tph[j] += t - tpl;
      tpl = t;
    }
  };
  const int ngr = gb - ga, nblk = bb - ba, nel = eb - ea;
  if (ngr < 1 || ngr > kMaxSbGroups || ga < 0 || gb > v.ng || nblk < 1 || nblk > kMaxSbBlocks || ba < 0 ||
      bb > v.nb || nel < 1 || nel > kMaxSbElems || ea < 0 || eb > v.n) {
    if (lane == 0) atomicOr(v.err, 4);
    pos_nf = v.n;
    return __int_as_float(0x7fc00000);
  }
  // the superblock's group maps and starts, one trip
  glds_copy16(W.g, v.grp + ga, ngr * (int)(sizeof(GroupMap) / 16));
  glds_copy4(W.gs, v.gsg + ga, ngr + 1);
  glds_copy4(W.bs, v.bsg + ba, nblk + 1);
  __builtin_amdgcn_s_waitcnt(0);
  if (stamp) W.tclk[1] = (long long)__builtin_amdgcn_s_memtime();
  phase(0);
  int q0 = 0;
  while (q0 < ngr) {
    const int qf = spec_walk<GroupMap>(s, W.g + q0, ngr - q0, kGroupM);
    phase(1);
    ws.g += qf;
    ws.gh += qf;
    const int q = q0 + qf;
    if (stamp && q0 == 0) W.tclk[2] = (long long)__builtin_amdgcn_s_memtime();
    if (q >= ngr) break;
    if (qf == min(kWalkC, ngr - q0)) {  // a full chunk verified: the next one
      q0 = q;
      continue;
    }
    // group q by its leaves (block indices relative to ba): its leaf maps
    // and elements, one trip
    ++ws.g;
    const int b0 = uni(W.gs[q]) - ba, b1 = uni(W.gs[q + 1]) - ba;
    if (b1 - b0 < 1 || b1 - b0 > 2 * kGW - 1 || b0 < 0 || b1 > nblk) {
      if (lane == 0) atomicOr(v.err, 8);
      pos_nf = v.n;
      return __int_as_float(0x7fc00000);
    }
    const int nbl = b1 - b0;
    const int ga0 = uni(W.bs[b0]), gb0 = uni(W.bs[b1]);  // the group's elements [ga0, gb0)
    if (gb0 - ga0 < 1 || gb0 - ga0 > kGrpElems || ga0 < ea || gb0 > eb) {
      if (lane == 0) atomicOr(v.err, 16);
      pos_nf = v.n;
      return __int_as_float(0x7fc00000);
    }
    const int e4 = ga0 & ~3, xo = ga0 - e4;
#if RST_SQ_GROUP_SERIAL
    (void)nbl;
    glds_copy16(W.x, v.X + e4, (gb0 - e4 + 3) >> 2);
    __builtin_amdgcn_s_waitcnt(0);
    if (stamp && q0 == 0) W.tclk[3] = (long long)__builtin_amdgcn_s_memtime();
    phase(2);
    ws.ser += 1;
    serial_adds(s, W.x + xo, gb0 - ga0);
    phase(4);
    if (!isfinite(s)) {
      pos_nf = (int64_t)gb0;
      return s;
    }
    q0 = q + 1;
    continue;
#endif
    glds_copy16(W.l, v.leaf + ba + b0, nbl * (int)(sizeof(Leaf) / 16));
    glds_copy16(W.x, v.X + e4, (gb0 - e4 + 3) >> 2);
    __builtin_amdgcn_s_waitcnt(0);
    if (stamp && q0 == 0) W.tclk[3] = (long long)__builtin_amdgcn_s_memtime();
    phase(2);
    int l0 = 0;
    while (l0 < nbl) {
      const int lf = spec_walk<Leaf>(s, W.l + l0, nbl - l0, kLeafM);
      phase(3);
      ws.l += lf;
      ws.lh += lf;
      const int bl = l0 + lf;  // (relative to b0)
      if (stamp && q0 == 0 && l0 == 0) W.tclk[4] = (long long)__builtin_amdgcn_s_memtime();
      if (bl >= nbl) break;
      if (lf == min(kWalkC, nbl - l0)) {
        l0 = bl;
        continue;
      }
      // the block by the reference's own adds (serial_adds: r07b, half the
      // clocks of a v_readlane per element)
      ++ws.l;
      ++ws.ser;
      const int e0 = uni(W.bs[b0 + bl]) - ga0, e1 = uni(W.bs[b0 + bl + 1]) - ga0;
      if (e1 - e0 < 1 || e1 - e0 > 2 * kW - 1 || e0 < 0 || e1 > gb0 - ga0) {
        if (lane == 0) atomicOr(v.err, 16);
        pos_nf = v.n;
        return __int_as_float(0x7fc00000);
      }
      serial_adds(s, W.x + xo + e0, e1 - e0);
      if (stamp && q0 == 0 && l0 == 0) W.tclk[5] = (long long)__builtin_amdgcn_s_memtime();
      phase(4);
      if (!isfinite(s)) {
        pos_nf = (int64_t)ga0 + e1;
        return s;
      }
      l0 = bl + 1;
    }
    q0 = q + 1;
  }
  if (stamp) W.tclk[6] = (long long)__builtin_amdgcn_s_memtime();
  if (ph && lane == 0) W.tph[5] += (long long)__builtin_amdgcn_s_memtime() - tp0;
  return s;
}

template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}

// one superblock map in registers: lane r holds entry r, lanes < kWalkC
// the header of superblock (chunk start + lane)
struct SbRegs {
  float E[kWalkC];
  int LO[kWalkC], HI[kWalkC];
  float G;
  int e0, m, fl;
  int ga, gb, ba, bb, ea, eb;  // lane q: superblock q's ranges (the descent's loads)
};

__device__ __forceinline__ void sb_fetch(const SbMap* __restrict__ sbm_, int nk, int k0, int lane,
                                         SbRegs& R) {
  // (global address space: generic loads would also count on lgkmcnt and
  // serialise with every LDS / scalar wait of the walk)
  const auto* sbm = gptr(sbm_);
#pragma unroll
  for (int q = 0; q < kWalkC; ++q) {
    const int k = min(k0 + q, nk - 1);  // (clamped: a step past the end is never taken)
    R.E[q] = sbm[k].e[lane].E;
    R.LO[q] = sbm[k].e[lane].LOu;
    R.HI[q] = sbm[k].e[lane].HIu;
  }
  const int kh = min(k0 + (lane & (kWalkC - 1)), nk - 1);
  R.G = sbm[kh].h.G;
  R.e0 = sbm[kh].h.e0;
  R.m = sbm[kh].h.m;
  R.fl = sbm[kh].h.flags;
  R.ga = sbm[kh].ga;
  R.gb = sbm[kh].gb;
  R.ba = sbm[kh].ba;
  R.bb = sbm[kh].bb;
  R.ea = sbm[kh].ea;
  R.eb = sbm[kh].eb;
}

__device__ __forceinline__ void sq_walk_body(const SqView& v, float* __restrict__ out, const int c) {
  RST_TL(v.tl, v.it, 5);
  __shared__ WalkLds W;
  const int lane = threadIdx.x;
  const SbMap* sbm = v.sbm + (int64_t)c * v.nk;
  const float* X = v.soa + (int64_t)c * v.ns;
  int* st = v.stats ? v.stats + c * 8 : nullptr;
  const uint64_t t0 = st ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t rt0 = st ? __builtin_amdgcn_s_memrealtime() : 0;  // (100 MHz: calibrates the clocks)
  if (lane == 0) {
    W.ws = WalkStats{0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < 8; ++j) W.tclk[j] = 0;
    for (int j = 0; j < 6; ++j) W.tph[j] = 0;
    W.tph_on = st != nullptr;
    W.pos_nf = -1;
  }
  __syncthreads();
  __shared__ MapEnt CE[kWalkC][kWave];  // the chunk's entries, for the checks
  int nsb = 0, nsbh = 0;
  float s = v.s0 ? v.s0[c] : 0.0f;  // (a stretch: the chain's value at its start)
  bool nf = false;  // s became non-finite (W.pos_nf)
  int k = 0;
  SbRegs cur, nxt;
  if (v.nk > 0) sb_fetch(sbm, v.nk, 0, lane, cur);
  uint64_t wait_clk = 0;
  while (k < v.nk && !nf) {
    if (st) {  // (statistics: the time waiting for this chunk's maps)
      const uint64_t ta = __builtin_amdgcn_s_memtime();
      const int j = k / kWalkC;
      (void)j;
      __builtin_amdgcn_s_waitcnt(0);
      wait_clk += __builtin_amdgcn_s_memtime() - ta;
    }
    // the next chunk in flight while this one is walked
    sb_fetch(sbm, v.nk, k + kWalkC, lane, nxt);
    k = __builtin_amdgcn_readfirstlane(k);  // (uniform: keep the chunk's bounds scalar)
    const int qn = min(kWalkC, v.nk - k);
#pragma unroll
    for (int q = 0; q < kWalkC; ++q) CE[q][lane] = MapEnt{cur.E[q], cur.LO[q], cur.HI[q]};
    // lane q: superblock k + q's header terms
    const int gbl = (int)__float_as_uint(cur.G);
    const int sgl = gbl >> 31;  // 0, or -1 for a negative G
    const int mkl = ((1 << (cur.m & 7)) - 1) & (kWave - 1);
    // The chunk's steps, speculatively and unchecked: lane q's input from
    // the steps before it composed as a parallel prefix (affine_hist: the
    // offset units from the bits of s and G, s - G in G's grid when both
    // share sign and binade; the residue's end E_r + du 2^e0 in E_r's bits);
    // s before step q is lane q of `hist`, lane qn the chunk's end.
    const int ql = min(lane, kWalkC - 1);
    const int sb0 = __builtin_amdgcn_readfirstlane((int)__float_as_uint(s));
    float El = CE[ql][0].E;
    int hist = affine_hist(sb0, (int)__float_as_uint(El), step_shift(El, cur.e0), gbl, 0, qn);
    if (__ballot(lane < qn && mkl != 0) != 0) {  // (a map with several residues: again with each lane's)
      const int rl = (((hist - gbl) ^ sgl) - sgl) & mkl;
      El = CE[ql][rl].E;
      hist = affine_hist(sb0, (int)__float_as_uint(El), step_shift(El, cur.e0), gbl, rl, qn);
    }
    s = __int_as_float(__builtin_amdgcn_readlane(hist, qn));
    // The checks, step q on lane q: s and G share sign and binade (else the
    // offset above is meaningless; G's grid is 2^e0, zero and subnormal G
    // included, so the bits differ by the offset in units), the map is usable, the
    // offset lies in the residue's window, E_r + du 2^e0 is exact
    // (Fast2Sum) and is what the step produced.
    const int nxb = __builtin_amdgcn_update_dpp(0, hist, 0x130, 0xf, 0xf, false);  // wave_shl:1: lane q <- q + 1
    int okl;
    {
      const int kk = ((hist - gbl) ^ sgl) - sgl;
      const int r = kk & mkl;
      const MapEnt en = CE[min(lane, kWalkC - 1)][r];
      const int du = kk - r;
      const float a = en.E, b = -ldexpf((float)(r - kk), cur.e0);
      const float o = en.E - ldexpf((float)(r - kk), cur.e0);
      const bool abig = fabsf(a) >= fabsf(b);
      const float big = abig ? a : b, sml = abig ? b : a;
      okl = (lane < qn) & ((((uint32_t)hist ^ (uint32_t)gbl) >> 23) == 0u) &
            ((cur.fl & kOpaque) == 0) & ((unsigned)cur.m <= (unsigned)kSbM) & (en.LOu <= du) & (du <= en.HIu) &
            ((o - big) == sml) & ((int)__float_as_uint(o) == nxb);
    }
    const uint64_t bad = __ballot(!okl) & ((1ull << kWalkC) - 1);
    int qf = kWalkC;
    if (bad != 0) {
      qf = (int)__builtin_ctzll(bad);
      s = __int_as_float(__builtin_amdgcn_readlane(hist, qf));
    }
    nsb += qf;
    nsbh += qf;
    if (qf == kWalkC) {
      k += kWalkC;
      cur = nxt;
      continue;
    }
    k += qf;
    if (k >= v.nk) break;
    // (rare) superblock k by its map's slow path or its groups, then a
    // fresh chunk from k + 1
    // (its map with the slow offset -- s in another binade than G -- from
    // the chunk's registers and LDS copy, then the descent)
    ++nsb;
    MapHdr h;
    h.G = __int_as_float(__builtin_amdgcn_readlane(gbl, qf));
    h.e0 = __builtin_amdgcn_readlane(cur.e0, qf);
    h.m = __builtin_amdgcn_readlane(cur.m, qf);
    h.flags = __builtin_amdgcn_readlane(cur.fl, qf);
    if (walk_try(s, h, CE[qf], kSbM)) {
      ++nsbh;
    } else {
      const DescArgs da{v.grp + (int64_t)c * v.ng, v.leaf + (int64_t)c * v.nb, v.bs + (int64_t)c * (v.nb + 1),
                        v.gs + (int64_t)c * (v.ng + 1), X, v.err, v.n, v.nb, v.ng};
      s = walk_descend(da, __builtin_amdgcn_readlane(cur.ga, qf), __builtin_amdgcn_readlane(cur.gb, qf),
                       __builtin_amdgcn_readlane(cur.ba, qf), __builtin_amdgcn_readlane(cur.bb, qf),
                       __builtin_amdgcn_readlane(cur.ea, qf), __builtin_amdgcn_readlane(cur.eb, qf), s, W);
      nf = W.pos_nf >= 0;
    }
    ++k;
    sb_fetch(sbm, v.nk, k, lane, cur);  // (unconditional: cur is dead across the descent)
  }
  if (nf) {
    // inf / NaN absorbs every finite element: only NaN or an opposite
    // infinity later can still change it.  Serial to the next window, then
    // the window flags.
    int64_t i = W.pos_nf;
    for (; i < v.n && (i % kW) != 0; ++i) s = s + X[i];
    int orf = 0;
    const uint8_t* wf = v.wflg + (int64_t)c * v.nb;
    for (int64_t w = i / kW + lane; w < v.nb; w += kWave) orf |= wf[w];
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) orf |= __shfl_xor(orf, o, kWave);
    if (isnan(s) || (orf & 1) || (s > 0 && (orf & 4)) || (s < 0 && (orf & 2))) s = __int_as_float(0x7fc00000);
  }
  if (lane == 0) {
    out[c] = s;
    // every chain reads err after its own walk: its descents' trips and the
    // map kernels' (an atomic read: the trips are L2 atomics)
    if (g_sq_fault) atomicOr(v.err, g_sq_fault);
    const int ev = atomicOr(v.err, 0);
    if (ev && v.guard) atomicOr(v.guard, kGuardSeqsum | (ev << kGuardSeqsumShift));
    if (c == 0 && v.stats) v.stats[32] = ev;
    if (st) {
      st[0] = nsb;
      st[1] = nsbh;
      st[2] = W.ws.g;
      st[3] = W.ws.gh;
      st[4] = W.ws.l;
      st[5] = W.ws.lh;
      st[6] = W.ws.ser;
      st[7] = (int)min<uint64_t>(INT_MAX, __builtin_amdgcn_s_memtime() - t0);
      if (c < 4) v.stats[c < 3 ? 37 + c : 56] = (int)min<uint64_t>(INT_MAX, __builtin_amdgcn_s_memrealtime() - rt0);
      if (c < 2)
        for (int j = 0; j < 6; ++j) v.stats[40 + 6 * c + j] = (int)min<long long>(INT_MAX, W.tph[j]);
      if (c < 4) v.stats[33 + c] = (int)min<uint64_t>(INT_MAX, wait_clk);
      if (c == 0)
        for (int j = 1; j < 7; ++j) v.stats[56 + j] = W.tclk[j] ? (int)(W.tclk[j] - W.tclk[0]) : -1;
    }
  }
}

// ---- the kernels: one stream (SqView by value), or a batch of streams -----------
__global__ __launch_bounds__(kFrontT) void k_sq_tot(const float4* __restrict__ x, SqView v) {
  sq_tot_body(x, v, blockIdx.x);
}
template <bool FUSED>
__global__ __launch_bounds__(kFrontT) void k_sq_front(SqView v, const float4* __restrict__ x,
                                                     const double* __restrict__ tprev,
                                                     double* __restrict__ tnext) {
  sq_front_body<FUSED>(v, x, tprev, tnext, blockIdx.x, blockIdx.y);
}
// the single-stream maps (a pair alone: latency) in one kernel -- the leaf
// runs, then wavefront 0 composes from the LDS copy; r20: split in two
// launches, a lone pair's maps 39 -> 50 us an iteration
__global__ __launch_bounds__(kBuildT1) void k_sq_build(SqView v) {
  __shared__ LeafLds WL;
  __shared__ CompLds WC;
  sq_leaf_body<kBuildT1>(v, blockIdx.x, blockIdx.y, WL, true);
  __syncthreads();
  if (threadIdx.x >= kWave) return;
  sq_comp_body(v, blockIdx.x, blockIdx.y, WC, WL.lf);
}
__global__ __launch_bounds__(kWave) void k_sq_walk(SqView v, float* __restrict__ out) {
  sq_walk_body(v, out, blockIdx.x);
}

// A batch of streams (the batched ICP loop, icp.hip): stream = blockIdx.z,
// its tables from a device array of SqPair records (seqsum_pair_fill); the
// grids fit the batch's longest stream, the other streams' extra blocks
// return at once.  nch and iter are the launch's (the records are laid out
// for 4 chains).
struct SqPair {
  const float4* x;
  float* out;
  SqView v;
};
// (every table pointer read back as a global pointer: as_glb, rst_device.hpp
// -- loaded from the SqPair array they were generic, and the batched
// kernels' accesses flat)
__device__ __forceinline__ SqView sq_at(const SqPair& P, int nch, int iter) {
  SqView v = P.v;
  v.soa = as_glb(P.v.soa);
  v.wflg = as_glb(P.v.wflg);
  v.bs = as_glb(P.v.bs);
  v.gs = as_glb(P.v.gs);
  v.ks = as_glb(P.v.ks);
  v.inc = as_glb(P.v.inc);
  v.ipre = as_glb(P.v.ipre);
  v.tinc = as_glb(P.v.tinc);
  v.leaf = as_glb(P.v.leaf);
  v.grp = as_glb(P.v.grp);
  v.sbm = as_glb(P.v.sbm);
  v.stats = as_glb(P.v.stats);
  v.ttot = as_glb(P.v.ttot);
  v.ttot2 = as_glb(P.v.ttot2);
  v.clk = as_glb(P.v.clk);
  v.err = as_glb(P.v.err);
  v.p0 = as_glb(P.v.p0);
  v.s0 = as_glb(P.v.s0);
  v.tl = as_glb(P.v.tl);
  v.guard = as_glb(P.v.guard);
  v.nch = nch;
  v.it = iter;
  if (iter >= 0) v.ttot = v.ttot2 + (size_t)(iter & 1) * 4 * kTotQ * v.nk;
  return v;
}
__global__ __launch_bounds__(kFrontT) void k_sq_tot_b(const SqPair* __restrict__ P, int nch, int iter) {
  const SqPair& p = P[blockIdx.z];
  const SqView v = sq_at(p, nch, iter);
  if ((int)blockIdx.x >= v.nk * kTotQ) return;
  sq_tot_body(as_glb(p.x), v, blockIdx.x);
}
template <bool FUSED>
__global__ __launch_bounds__(kFrontT) void k_sq_front_b(const SqPair* __restrict__ P, int nch, int iter) {
  const SqPair& p = P[blockIdx.z];
  const SqView v = sq_at(p, nch, iter);
  if ((int)blockIdx.x >= v.nk) return;
  if constexpr (FUSED) {  // (iter >= 1: the previous iteration's totals by parity)
    const double* tprev = v.ttot2 + (size_t)((iter - 1) & 1) * 4 * kTotQ * v.nk;
    sq_front_body<true>(v, as_glb(p.x), tprev, v.ttot, blockIdx.x, blockIdx.y);
  } else {
    sq_front_body<false>(v, nullptr, nullptr, nullptr, blockIdx.x, blockIdx.y);
  }
}
__global__ __launch_bounds__(kBuildT, kLeavesWaves) void k_sq_leaves_b(const SqPair* __restrict__ P, int nch, int iter) {
  const SqView v = sq_at(P[blockIdx.z], nch, iter);
  if ((int)blockIdx.x >= v.nk) return;
  __shared__ LeafLds W;
  sq_leaf_body<kBuildT>(v, blockIdx.x, blockIdx.y, W, false);
}
__global__ __launch_bounds__(kWave) void k_sq_comp_b(const SqPair* __restrict__ P, int nch, int iter) {
  const SqView v = sq_at(P[blockIdx.z], nch, iter);
  if ((int)blockIdx.x >= v.nk) return;
  __shared__ CompLds W;
  sq_comp_body(v, blockIdx.x, blockIdx.y, W, nullptr);
}
__global__ __launch_bounds__(kWave) void k_sq_walk_b(const SqPair* __restrict__ P, int nch, int iter) {
  const SqPair& p = P[blockIdx.z];
  const SqView v = sq_at(p, nch, iter);
  sq_walk_body(v, as_glb(p.out), blockIdx.x);
}


// ---- 5: small streams, one workgroup per chain -----------------------------------
// Streams of <= kSmallMax elements (the reference callers' 5 cm clouds,
// ~15k points, rs_replay_app.cpp:246-251) take the map pipeline's whole
// statement on one CU per chain, in one launch: the chain's elements staged
// in LDS (padded 17 words per 16), a thread per 16-element window -- the
// window's fp64 total, block scan, the block start at the largest |prefix|
// among window positions [kJLo, kJHi] (the front's rule), the block's
// unmonitored float run from its fp64 guess and a scan of those increments
// (the drift-corrected guesses), then candidate 0's monitored run (extra
// candidates listed, one lane each) -- every leaf map in LDS; group maps
// over 16-block windows (lattice, (group, candidate) composites, the big
// kernel's branch-free steps); then wavefront 0 walks the <= 64 group maps
// (spec_walk), descending to a group's leaf maps and a block's own adds.
// No global tables, no bound checks that can trip: sizes are the launch's.
// A chain with a non-finite element is replayed by wavefront 0 (the
// reference loop itself). r10: the pipeline's five launches cost ~50-65 us
// an iteration at these sizes whatever the length.
constexpr int kSmT = 1024;             // threads: one 16-element window each
constexpr int kSmallMax = kSmT * kW;   // 16384 elements
constexpr int kSmGroups = kSmT / kGW;  // 64 group windows
constexpr int kSmXs = kSmallMax + 2 * kW;
constexpr int kSmXsPad = kSmXs + kSmXs / kW;
constexpr int kSmList = (kLeafR - 1) * kSmT;
struct GroupMapS {  // a group map without the global layout's padding
  MapHdr h;
  MapEnt e[kGroupR];
};
struct SmallLds {
  float xs[kSmXsPad];            // the chain's elements, xs(i) at i + i / 16 (the walk's own
                                 // adds read them too: r10a, from global memory, ~60 us a call)
  Leaf lf[kSmT];
  union {
    int16_t xneed[kSmT][kLeafR - 1];  // the leaves' extra candidates' needs (leaf phase)
    GroupMapS gm[kSmGroups];          // the group maps (group phase on)
  } u;
  int bst[kSmT + 1];             // block starts (elements)
  int gst[kSmGroups + 1];        // group starts (blocks)
  int8_t gexact[kSmGroups];      // a group's lattice beyond kGroupM: exact-only windows
  uint16_t list[kSmList];        // the leaves' extra candidates, then the groups'
  double scan[kSmT / kWave + 1];
  int nlist, ngr;
};
static_assert(sizeof(SmallLds) <= 160 * 1024, "small-stream LDS");

__device__ __forceinline__ float& sm_x(SmallLds& W, int i) { return W.xs[i + (i >> 4)]; }

// s <- the reference's adds over elements [a, a + cnt) of the padded LDS copy
// (serial_adds' rounds: 32 broadcast reads, then 32 dependent adds; +0 past cnt)
__device__ __forceinline__ void serial_adds_sm(float& s, SmallLds& W, int a, int cnt) {
  constexpr int kR = 32;
  cnt = __builtin_amdgcn_readfirstlane(cnt);
  a = __builtin_amdgcn_readfirstlane(a);
  for (int c0 = 0; c0 < cnt; c0 += kR) {
    float xr[kR];
#pragma unroll
    for (int i = 0; i < kR; ++i) xr[i] = c0 + i < cnt ? sm_x(W, a + c0 + i) : 0.0f;
#pragma unroll
    for (int i = 0; i < kR; ++i) s = s + xr[i];
  }
}

__global__ __launch_bounds__(kSmT) void k_sq_small(const float4* __restrict__ x, int64_t n64, int nch,
                                                   const double* __restrict__ p0, const float* __restrict__ s0,
                                                   float* __restrict__ out, int* __restrict__ guard,
                                                   int* __restrict__ stats) {
  __shared__ SmallLds W;
  // (diagnostics, rst_debug_seq_sum's stats: chain 0's phase clocks and walk
  // counts -- group tries / hits, leaf tries / hits, blocks added serially)
  const bool stm = stats && blockIdx.x == 0 && threadIdx.x == 0;
  const long long ck0 = stm ? (long long)__builtin_amdgcn_s_memtime() : 0;
  auto mark = [&](int j) {
    if (stm) stats[j] = (int)((long long)__builtin_amdgcn_s_memtime() - ck0);
  };
  const int c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int n = (int)n64;
  if (c >= nch) return;
  if (tid == 0) W.nlist = 0;
  // -- the elements, coalesced float4 loads, component c into LDS (every
  // load issued before the first store: r10b, a load-store pair per element
  // waited out a memory round trip each, ~30 us at any length)
  constexpr int kLd = kSmXs / kSmT + 1;
  float tv[kLd];
#pragma unroll
  for (int k = 0; k < kLd; ++k) {
    const int i = tid + k * kSmT;
    tv[k] = i < n ? comp(x[i], c) : 0.0f;
  }
  int fl = 0;
#pragma unroll
  for (int k = 0; k < kLd; ++k) {
    const int i = tid + k * kSmT;
    fl |= nf_flags(tv[k]);
    if (i < kSmXs) sm_x(W, i) = tv[k];
  }
  const float sst = s0 ? s0[c] : 0.0f;
  const bool anynf = __syncthreads_or(fl != 0 || !isfinite(sst));
  mark(0);
  if (anynf) {  // (inf / NaN: the reference's own adds, in order)
    if (tid < kWave) {
      float s = sst;
      for (int i0 = 0; i0 < n; i0 += 32) {
        float xr[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) xr[j] = i0 + j < n ? sm_x(W, i0 + j) : 0.0f;
#pragma unroll
        for (int j = 0; j < 32; ++j) s = s + xr[j];
      }
      if (tid == 0) out[c] = s;
    }
    return;
  }
  const double P = p0 ? p0[c] : 0.0;
  const int nb = (n + kW - 1) / kW;
  const bool act = tid < nb;
  // -- the window's fp64 total and prefix; the block start
  double wsum = 0.0;
#pragma unroll
  for (int j = 0; j < kW; ++j) wsum += (double)sm_x(W, tid * kW + j);  // (+0 past n)
  double ttot;
  const double wpre = P + block_scan_excl<kSmT>(act ? wsum : 0.0, W.scan, &ttot);
  double best = wpre, run = wpre;
  int bj = -1;
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    if (j >= kJLo && j <= kJHi && (bj < 0 || fabs(run) > fabs(best)) && tid * kW + j < n) {
      best = run;
      bj = j;
    }
    run += (double)sm_x(W, tid * kW + j);
  }
  if (bj < 0) {
    best = wpre;
    bj = 0;
  }
  if (tid == 0) {
    best = p0 ? P : 0.0;
    bj = 0;
  }
  if (act) W.bst[tid] = tid * kW + bj;
  if (tid == 0) W.bst[nb] = n;
  // group starts: the block of largest |start| among blocks [kJLo, kJHi] of
  // each 16-block window (the front's rule)
  {
    const int wj = tid & (kGW - 1);
    double key = act ? (wj >= kJLo && wj <= kJHi ? fabs(best) : -0.5) : -1.0;
    int kid = act ? tid : INT_MAX;
#pragma unroll
    for (int st = 0; st < 4; ++st) {  // (DPP, as the front kernel's)
      double ok;
      int oi;
      switch (st) {
        case 0: ok = dpp_d<kRowBfly[0]>(key); oi = dpp_i<kRowBfly[0]>(kid); break;
        case 1: ok = dpp_d<kRowBfly[1]>(key); oi = dpp_i<kRowBfly[1]>(kid); break;
        case 2: ok = dpp_d<kRowBfly[2]>(key); oi = dpp_i<kRowBfly[2]>(kid); break;
        default: ok = dpp_d<kRowBfly[3]>(key); oi = dpp_i<kRowBfly[3]>(kid); break;
      }
      if (ok > key || (ok == key && oi < kid)) {
        key = ok;
        kid = oi;
      }
    }
    const int q = tid / kGW;
    const int ngr = (nb + kGW - 1) / kGW;
    if ((tid & (kGW - 1)) == 0 && q < ngr) W.gst[q] = q == 0 ? 0 : kid;
    if (tid == 0) {
      W.gst[ngr] = nb;
      W.ngr = ngr;
    }
  }
  __syncthreads();
  mark(1);
  // -- the block's unmonitored run from its fp64 guess; the increments' scan
  const int a0 = act ? W.bst[tid] : 0;
  const int len = act ? W.bst[tid + 1] - a0 : 0;  // <= kW + kJHi - kJLo < 2 kW
  float w[2 * kW];
#pragma unroll
  for (int j = 0; j < 2 * kW; ++j) w[j] = j < len ? sm_x(W, a0 + j) : 0.0f;
  double incv = 0.0;
  {
    const float G0 = tid == 0 && !p0 ? 0.0f : (float)best;
    float sr = G0;
#pragma unroll
    for (int j = 0; j < 2 * kW; ++j)
      if (j < len) sr = sr + w[j];
    incv = act ? (double)sr - (double)G0 : 0.0;
  }
  double itot;
  const double ipre = block_scan_excl<kSmT>(incv, W.scan, &itot);
  // -- leaves: candidate 0, the block's guess
  const float G = candidate_base(tid == 0 && !p0 ? 0.0f : (float)(P + ipre), kLeafR);
  const int e0 = grid_exp(G);
  Run pr;
  run_init(pr, G);
  const int wmax = wave_max_small<5>(len);
#pragma unroll
  for (int j = 0; j < 2 * kW; ++j)
    if (j < wmax && j < len) run_step(pr, w[j], e0);
  const int m0 = pr.need == kNoNeed ? 0 : max(0, pr.need - e0);
  const bool more = act && !pr.opaque && m0 >= 1 && m0 <= kLeafM;
  if (act) W.lf[tid].h = MapHdr{G, e0, 0, 0};  // (the list lanes read G, e0)
  if (more) {
    const int at = atomicAdd(&W.nlist, kLeafR - 1);
#pragma unroll
    for (int r = 1; r < kLeafR; ++r) W.list[at + r - 1] = (uint16_t)(tid << 2 | r);  // (<= 3 per block)
  }
  __syncthreads();
  mark(2);
  {
    // the listed extra candidates, one lane each (rare; uniform skip)
    const int nl = W.nlist;
    for (int j0 = 0; j0 < nl; j0 += kSmT) {
      const int j = j0 + tid;
      const int code = j < nl ? W.list[j] : 0;
      const int bl = code >> 2, r = code & 3;
      const int xa = j < nl ? W.bst[bl] : 0, xl = j < nl ? W.bst[bl + 1] - xa : 0;
      const float xG = j < nl ? W.lf[bl].h.G : 0.0f;
      const int xe0 = j < nl ? W.lf[bl].h.e0 : -149;
      const int xw = wave_max_small<5>(xl);
      if (xw > 0) {
        float v[2 * kW];
#pragma unroll
        for (int q = 0; q < 2 * kW; ++q) v[q] = q < xl ? sm_x(W, xa + q) : 0.0f;
        Run q;
        run_init(q, cand(xG, xe0, r));
#pragma unroll
        for (int t = 0; t < 2 * kW; ++t)
          if (t < xw && t < xl) run_step(q, v[t], xe0);
        if (j < nl) {
          W.lf[bl].e[r] = leaf_ent(q, xe0);
          W.u.xneed[bl][r - 1] = q.need == kNoNeed ? kNeedNone : (int16_t)max(-32767, min(32767, q.need));
        }
      }
    }
  }
  __syncthreads();
  if (act) {
    int need = pr.need;
    if (more)
#pragma unroll
      for (int r = 1; r < kLeafR; ++r) {
        const int xn = W.u.xneed[tid][r - 1];
        need = max(need, xn == kNeedNone ? kNoNeed : xn);
      }
    const int mneed = need == kNoNeed ? 0 : max(0, need - e0);
    const bool exact_only = mneed > kLeafM;
    const int m = exact_only ? 0 : mneed;
    Leaf o;
    o.h = MapHdr{G, e0, m, pr.opaque ? kOpaque : 0};
    o.e[0] = leaf_ent(pr, e0);
#pragma unroll
    for (int r = 1; r < kLeafR; ++r) o.e[r] = more ? W.lf[tid].e[r] : MapEnt{0.0f, 1, 0};
#pragma unroll
    for (int r = 0; r < kLeafR; ++r) {
      if (r >= (1 << m)) {
        o.e[r].LOu = 1;
        o.e[r].HIu = 0;
      } else if (exact_only) {
        o.e[r].LOu = max(o.e[r].LOu, 0);
        o.e[r].HIu = min(o.e[r].HIu, 0);
      }
    }
    W.lf[tid] = o;
  }
  const int ngr = W.ngr;
  if (tid == 0) W.nlist = ngr;  // the group list: every group's candidate 0 first
  __syncthreads();
  mark(3);
  // -- groups (their maps take the leaves' needs' place)
  if (tid < ngr) {
    const int gi = tid;
    const int g0 = W.gst[gi], g1 = W.gst[gi + 1];
    GroupMapS& o = W.u.gm[gi];
    const MapHdr h0 = W.lf[g0].h;
    int lat = h0.e0 + h0.m;
    for (int j = g0 + 1; j < g1; ++j) {
      const MapHdr hj = W.lf[j].h;
      lat = (hj.flags & kOpaque) ? lat : max(lat, hj.e0 + hj.m);
    }
    int m = max(0, lat - h0.e0);
    const bool exact_only = m > kGroupM;
    if (exact_only) m = 0;
    const int R = 1 << m;
    const float Gg = candidate_base(h0.G, R);
    o.h = MapHdr{Gg, grid_exp(Gg), m, 0};
    W.gexact[gi] = exact_only ? 1 : 0;
    for (int r = 0; r < kGroupR; ++r) o.e[r] = MapEnt{0.0f, 1, 0};
    if (R > 1) {
      const int at = atomicAdd(&W.nlist, R - 1);
      for (int r = 1; r < R; ++r) W.list[at + r - 1] = (uint16_t)(gi << 4 | r);  // (<= 64 x 16)
    }
  }
  __syncthreads();
  {
    // lanes (group, candidate) through the group's leaf maps (the big
    // kernel's branch-free composite, sq_build_body)
    const int nl = W.nlist;  // <= kSmGroups x kGroupR = kSmT
    const int j = tid;
    if (j - lane < nl) {
      const bool ea_ = j < nl;
      const int code = !ea_ ? 0 : (j < ngr ? j << 4 : W.list[j]);
      const int gi = code >> 4, r = code & (kGroupR - 1);
      const int c0 = W.gst[gi], c1 = W.gst[gi + 1];
      const MapHdr gh = W.u.gm[gi].h;
      float xv = cand(gh.G, gh.e0, r);
      double clo = -INFINITY, chi = INFINITY;
      bool ok = ea_;
      const int4* lq = reinterpret_cast<const int4*>(W.lf);
      int4 q0 = lq[4 * c0], q1 = lq[4 * c0 + 1], q2 = lq[4 * c0 + 2], q3 = lq[4 * c0 + 3];
      const int nst = wave_max_small<5>(ea_ ? c1 - c0 : 0);  // (a group <= 2 kGW - 1 blocks)
      for (int st = 0; st < nst; ++st) {
        const int jl = c0 + st;
        const int jn = 4 * min(jl + 1, c1 - 1);
        const int4 n0 = lq[jn], n1 = lq[jn + 1], n2 = lq[jn + 2], n3 = lq[jn + 3];
        const MapHdr h{__int_as_float(q0.x), q0.y, q0.z, q0.w};
        bool okj = ok && jl < c1;
        const int kq = comp_off(xv, h, kLeafM, okj);
        const int rr = kq & ((1 << (okj ? h.m : 0)) - 1);
        const bool r0 = (rr & 1) != 0, r1 = (rr & 2) != 0;
        MapEnt en;
        en.E = __int_as_float(r1 ? (r0 ? q3.y : q2.z) : (r0 ? q1.w : q1.x));
        en.LOu = r1 ? (r0 ? q3.z : q2.w) : (r0 ? q2.x : q1.y);
        en.HIu = r1 ? (r0 ? q3.w : q3.x) : (r0 ? q2.y : q1.z);
        comp_apply(xv, clo, chi, okj, h, kq, en);
        ok = jl < c1 ? okj : ok;
        q0 = n0;
        q1 = n1;
        q2 = n2;
        q3 = n3;
      }
      if (ea_ && ok) {
        if (W.gexact[gi]) {
          clo = fmax(clo, 0.0);
          chi = fmin(chi, 0.0);
        }
        W.u.gm[gi].e[r] = MapEnt{xv, lo_units(clo, gh.e0), hi_units(chi, gh.e0)};
      }
    }
  }
  __syncthreads();
  mark(4);
  if (tid >= kWave) return;
  int ngt = 0, ngh = 0, nlt = 0, nlh = 0, nser = 0;
  // -- the walk: wavefront 0 over the group maps, a missed group by its leaf
  // maps, a missed block by its own adds
  float sv = sst;
  int q0 = 0;
  while (q0 < ngr) {
    const int qf = spec_walk<GroupMapS>(sv, W.u.gm + q0, ngr - q0, kGroupM);
    const int q = q0 + qf;
    ngt += min(qf + 1, ngr - q0);
    ngh += qf;
    if (q >= ngr) break;
    if (qf == min(kWalkC, ngr - q0)) {
      q0 = q;
      continue;
    }
    const int b0 = __builtin_amdgcn_readfirstlane(W.gst[q]), b1 = __builtin_amdgcn_readfirstlane(W.gst[q + 1]);
    int l0 = b0;
    while (l0 < b1) {
      const int lf = spec_walk<Leaf>(sv, W.lf + l0, b1 - l0, kLeafM);
      const int bl = l0 + lf;
      nlt += min(lf + 1, b1 - l0);
      nlh += lf;
      if (bl >= b1) break;
      if (lf == min(kWalkC, b1 - l0)) {
        l0 = bl;
        continue;
      }
      // block bl by the reference's adds (its elements in LDS)
      const int ea = __builtin_amdgcn_readfirstlane(W.bst[bl]);
      const int ln = __builtin_amdgcn_readfirstlane(W.bst[bl + 1]) - ea;
      serial_adds_sm(sv, W, ea, ln);
      ++nser;
      l0 = bl + 1;
    }
    q0 = q + 1;
  }
  mark(5);
  if (stm) {
    stats[8] = ngt;
    stats[9] = ngh;
    stats[10] = nlt;
    stats[11] = nlh;
    stats[12] = nser;
    stats[13] = ngr;
  }
  if (lane == 0) {
    out[c] = sv;
    if (g_sq_fault && guard) atomicOr(guard, kGuardSeqsum | (g_sq_fault << kGuardSeqsumShift));
  }
}
}  // namespace

// the workspace layout (seqsum_bytes sizes it for 4 chains)
static size_t sq_layout(SqView& v, int64_t n, int nch, char* base) {
  v.n = n;
  v.ns = (n + 63) & ~(int64_t)63;
  v.nch = nch;
  v.nb = (int)((n + kW - 1) / kW);
  v.ng = (v.nb + kGW - 1) / kGW;
  v.nk = (v.ng + kKW - 1) / kKW;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return q;
  };
  // (first: its place must not depend on nch -- consecutive calls with
  // different chain counts share it)
  v.ttot2 = (double*)take(sizeof(double) * 2 * 4 * 4 * (size_t)v.nk);
  v.soa = (float*)take(sizeof(float) * nch * (size_t)v.ns);
  v.wflg = (uint8_t*)take((size_t)nch * v.nb);
  v.err = (int*)take(sizeof(int));
  v.ttot = (double*)take(sizeof(double) * nch * 4 * (size_t)v.nk);
  v.bs = (int*)take(sizeof(int) * nch * (size_t)(v.nb + 1));
  v.gs = (int*)take(sizeof(int) * nch * (size_t)(v.ng + 1));
  v.ks = (int*)take(sizeof(int) * nch * (size_t)(v.nk + 1));
  v.inc = (double*)take(sizeof(double) * nch * (size_t)v.nb);
  v.ipre = (double*)take(sizeof(double) * nch * (size_t)v.nb);
  v.tinc = (double*)take(sizeof(double) * nch * (size_t)v.nk);
  v.leaf = (Leaf*)take(sizeof(Leaf) * nch * (size_t)v.nb);
  v.grp = (GroupMap*)take(sizeof(GroupMap) * nch * (size_t)v.ng);
  v.sbm = (SbMap*)take(sizeof(SbMap) * nch * (size_t)v.nk);
  v.clk = (long long*)take(sizeof(long long) * 8 * nch * (size_t)v.nk);
  return off;
}

size_t seqsum_bytes(int64_t n) {
  SqView v;
  return sq_layout(v, std::max<int64_t>(n, 1), 4, nullptr);
}

// out[c] for c < nch: the sequential float sum of component c of x[0..n).
// stages (debug): bit 0 the front kernel, bit 1 the maps, bit 2 the walk.
// iter >= 0 (an ICP loop's iteration on one workspace): the quarter totals
// go to the iteration's parity buffer; fused (iter > 0, the same chains as
// iteration iter - 1 summed on this workspace): no totals launch, the front
// kernel takes the tile prefixes of iteration iter - 1.
// the replay's ceiling (elements; RST_SQ_SERIAL_MAX: tuning knob, 0 = never)
static int64_t serial_max() {
  static const int64_t g = [] {
    const char* e = getenv("RST_SQ_SERIAL_MAX");
    const long long v = e ? atoll(e) : (long long)kSerDefault;
    return (int64_t)(v < 0 ? 0 : v);
  }();
  return g;
}

// the one-workgroup-per-chain kernel's ceiling (elements; RST_SQ_SMALL_MAX:
// tuning knob, 0 = never; at most kSmallMax)
static int64_t small_max() {
  static const int64_t g = [] {
    const char* e = getenv("RST_SQ_SMALL_MAX");
    const long long v = e ? atoll(e) : (long long)kSmallMax;
    return (int64_t)(v < 0 ? 0 : std::min<long long>(v, kSmallMax));
  }();
  return g;
}

namespace {
// a stretch's chain totals: the quarter tiles' fp64 totals (k_sq_tot), per
// chain in a fixed order (block 0 of the relay's exchange)
__global__ __launch_bounds__(kFrontT) void k_sq_sumq(SqView v, double* __restrict__ tot4) {
  __shared__ double lds[kFrontT / kWave + 1];
  for (int c = 0; c < 4; ++c) {
    double t = 0.0;
    if (c < v.nch) t = block_sum_global<kFrontT>(v.ttot + (int64_t)c * v.nk * kTotQ, v.nk * kTotQ, lds);
    if (threadIdx.x == 0) tot4[c] = t;
    __syncthreads();
  }
}
__global__ void k_sq_copy4(const float* __restrict__ s0, int nch, float* __restrict__ out) {
  if ((int)threadIdx.x < nch) out[threadIdx.x] = s0 ? s0[threadIdx.x] : 0.0f;
}
}  // namespace

size_t seqsum_pair_bytes() { return sizeof(SqPair); }

void seqsum_pair_fill(void* rec, const float4* d_x, int64_t n, void* ws, float* d_out, unsigned long long* tl,
                      int* d_guard) {
  SqPair p;
  p.x = d_x;
  p.out = d_out;
  sq_layout(p.v, std::max<int64_t>(n, 1), 4, (char*)ws);
  p.v.n = n;
  p.v.guard = d_guard;
  p.v.stats = nullptr;
  p.v.p0 = nullptr;
  p.v.s0 = nullptr;
  p.v.tl = tl;
  p.v.it = -1;
  memcpy(rec, &p, sizeof(p));
}

// (measured r08: the batched value 26.4k fused vs 26.9k not -- a one-batch
// iteration's sums 266 vs 227 us; the fused front redoes the quarter totals
// once per chain: off)
#ifndef RST_SQ_FUSE_BATCH
#define RST_SQ_FUSE_BATCH 0
#endif
int seqsum_enqueue_batch(const void* d_pairs, int nbatch, int64_t nmax, int nch, int iter, hipStream_t st,
                         int nch_prev) {
  if (nch < 1 || nch > 4 || nbatch < 1 || nmax < 1 || nmax > (int64_t)INT_MAX - 2 * kTile) return RST_E_ARG;
  const int nb = (int)((nmax + kW - 1) / kW), ng = (nb + kGW - 1) / kGW, nk = (ng + kKW - 1) / kKW;
  const SqPair* P = (const SqPair*)d_pairs;
  // (fused: an iteration after the first whose chains the previous one ran
  // too -- not the last, which adds the cost chain -- takes its tile
  // prefixes from the previous iteration's totals, no k_sq_tot_b launch)
  if (RST_SQ_FUSE_BATCH && iter >= 1 && nch == 3 && nch_prev == 3) {
    k_sq_front_b<true><<<dim3(nk, nch, nbatch), kFrontT, 0, st>>>(P, nch, iter);
  } else {
    k_sq_tot_b<<<dim3(nk * kTotQ, 1, nbatch), kFrontT, 0, st>>>(P, nch, iter);
    k_sq_front_b<false><<<dim3(nk, nch, nbatch), kFrontT, 0, st>>>(P, nch, iter);
  }
  k_sq_leaves_b<<<dim3(nk, nch, nbatch), kBuildT, 0, st>>>(P, nch, iter);
  k_sq_comp_b<<<dim3(nk, nch, nbatch), kWave, 0, st>>>(P, nch, iter);
  k_sq_walk_b<<<dim3(nch, 1, nbatch), kWave, 0, st>>>(P, nch, iter);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

namespace {
// (test hook: the DPP scans on one wave of given values, rst_debug_wave_scan)
__global__ __launch_bounds__(kWave) void k_wave_scan_test(const double* __restrict__ in, double* __restrict__ out) {
  __shared__ double lds[kWave];
  const int t = threadIdx.x;
  out[t] = wave_scan_incl(in[t]);
  double tot;
  const double ex = block_scan_excl<kWave>(in[kWave + t], lds, &tot);
  out[kWave + t] = ex;
  if (t == 0) out[2 * kWave] = tot;
}
}  // namespace

int seqsum_debug_wave_scan(hipStream_t st, const double* h_in, double* h_out) {
  double* d = nullptr;
  if (hipMalloc(&d, sizeof(double) * (4 * kWave + 1)) != hipSuccess) return RST_E_NOMEM;
  int rc = RST_OK;
  if (hipMemcpyAsync(d, h_in, sizeof(double) * 2 * kWave, hipMemcpyHostToDevice, st) != hipSuccess) rc = RST_E_HIP;
  if (rc == RST_OK) {
    k_wave_scan_test<<<1, kWave, 0, st>>>(d, d + 2 * kWave);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(h_out, d + 2 * kWave, sizeof(double) * (2 * kWave + 1), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      rc = RST_E_HIP;
  }
  (void)hipFree(d);
  return rc;
}

int seqsum_debug_fault(int bits) {
  RST_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sq_fault), &bits, sizeof(int)));
  return RST_OK;
}

int seqsum_totals(const float4* d_x, int64_t n, int nch, void* ws, double* d_tot4, hipStream_t st, int iter) {
  if (nch < 1 || nch > 4 || n < 0) return RST_E_ARG;
  if (n == 0) {
    RST_HIP(hipMemsetAsync(d_tot4, 0, sizeof(double) * 4, st));
    return RST_OK;
  }
  if (n > (int64_t)INT_MAX - 2 * kTile) return RST_E_ARG;
  SqView v;
  sq_layout(v, n, nch, (char*)ws);
  v.stats = nullptr;
  v.p0 = nullptr;
  v.s0 = nullptr;
  v.tl = nullptr;
  v.it = iter;
  v.guard = nullptr;
  const size_t tq = (size_t)4 * kTotQ * v.nk;
  if (iter >= 0) v.ttot = v.ttot2 + (size_t)(iter & 1) * tq;
  k_sq_tot<<<v.nk * kTotQ, kFrontT, 0, st>>>(d_x, v);
  k_sq_sumq<<<1, kFrontT, 0, st>>>(v, d_tot4);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int seqsum_enqueue(const float4* d_x, int64_t n, int nch, void* ws, float* d_out, hipStream_t st,
                   int* d_stats, int stages, int iter, bool fused, const SqStretch* stretch,
                   unsigned long long* tl, int* d_guard) {
  if (nch < 1 || nch > 4 || n < 0) return RST_E_ARG;
  const float* s0 = stretch ? stretch->s0 : nullptr;
  if (n == 0) {  // (a stretch: the chain's value at its start, unchanged)
    k_sq_copy4<<<1, kWave, 0, st>>>(s0, nch, d_out);
    RST_HIP(hipGetLastError());
    return RST_OK;
  }
  if (n > (int64_t)INT_MAX - 2 * kTile) return RST_E_ARG;
  // short streams: one wavefront replays the chains; small ones: a
  // workgroup per chain maps and walks its chain on one CU (the whole sum in
  // one launch, no stats)
  const bool whole = (stages & 7) == 7;
  const bool forced = (stages & (kSqForceMaps | kSqForceSerial | kSqForceSmall)) != 0;
  if (whole && ((stages & kSqForceSerial) || (!forced && n <= serial_max()))) {
    k_sq_serial<<<1, kWave, 0, st>>>(d_x, n, nch, s0, d_out);
    RST_HIP(hipGetLastError());
    return RST_OK;
  }
  if (whole && n <= kSmallMax && ((stages & kSqForceSmall) || (!forced && n <= small_max()))) {
    // (its own stats layout -- phase clocks, group / leaf counts -- only for
    // rst_debug_seq_sum's forced path; the loop's per-chain walk stats stay
    // zero for such chains, rst_debug.h)
    k_sq_small<<<nch, kSmT, 0, st>>>(d_x, n, nch, stretch ? stretch->p0 : nullptr, s0, d_out, d_guard,
                                     (stages & kSqForceSmall) ? d_stats : nullptr);
    RST_HIP(hipGetLastError());
    return RST_OK;
  }
  stages &= 7;
  SqView v;
  sq_layout(v, n, nch, (char*)ws);
  v.stats = d_stats;
  v.p0 = stretch ? stretch->p0 : nullptr;
  v.s0 = s0;
  v.tl = tl;
  v.it = iter;
  v.guard = d_guard;
#ifdef RST_SQ_ABLATE  // measurement only (wrong sums): skip kernels by bit
  stages &= ~RST_SQ_ABLATE;
#endif
  const size_t tq = (size_t)4 * kTotQ * v.nk;  // one parity buffer: 4 chains' quarter totals
  if (iter >= 0) v.ttot = v.ttot2 + (size_t)(iter & 1) * tq;
  if (stages & 1) {
    if (fused && iter > 0 && !stretch) {
      k_sq_front<true><<<dim3(v.nk, nch), kFrontT, 0, st>>>(v, d_x, v.ttot2 + (size_t)((iter - 1) & 1) * tq,
                                                            v.ttot);
    } else {
      // (a stretch's totals are in place: seqsum_totals ran for the exchange)
      if (!(stretch && stretch->tot_done)) k_sq_tot<<<v.nk * kTotQ, kFrontT, 0, st>>>(d_x, v);
      k_sq_front<false><<<dim3(v.nk, nch), kFrontT, 0, st>>>(v, nullptr, nullptr, nullptr);
    }
  }
  if (stages & 2) k_sq_build<<<dim3(v.nk, nch), kBuildT1, 0, st>>>(v);
  if (stages & 4) k_sq_walk<<<nch, kWave, 0, st>>>(v, d_out);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

}  // namespace rst
