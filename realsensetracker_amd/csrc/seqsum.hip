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
  double* tinc;    // [nch][nk]
  Leaf* leaf;      // [nch][nb]
  GroupMap* grp;   // [nch][ng]
  SbMap* sbm;      // [nch][nk]
  int* stats;      // optional, 8 per chain
  double* ttot;    // [nch][nk] fp64 tile totals
  int* err;        // bound-check failures (bits; 0 = none): a map kernel that
                   // meets a size its tables cannot hold stops instead of
                   // reading out of range
};

__device__ __forceinline__ float comp(const float4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ int nf_flags(float x) {
  if (isnan(x)) return 1;
  if (isinf(x)) return x > 0 ? 2 : 4;
  return 0;
}

// exclusive block scan of one double per thread (BS threads); returns the
// prefix, *total = the block total
template <int BS>
__device__ double block_scan_excl(double v, double* lds, double* total) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  double inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  if (lane == kWave - 1) lds[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int i = 0; i < BS / kWave; ++i) {
      const double t = lds[i];
      lds[i] = a;
      a += t;
    }
    lds[BS / kWave] = a;
  }
  __syncthreads();
  const double r = lds[w] + inc - v;
  *total = lds[BS / kWave];
  __syncthreads();
  return r;
}

// sum of a[0..cnt) (doubles, global) over the block, fixed order per thread
template <int BS>
__device__ double block_sum_global(const double* a, int cnt, double* lds) {
  double s = 0.0;
  for (int i = threadIdx.x; i < cnt; i += BS) s += a[i];
  double tot;
  (void)block_scan_excl<BS>(s, lds, &tot);
  return tot;
}

// ---- 1: SoA copy, window flags, fp64 tile totals --------------------------------
// One 4096-element tile per workgroup, 16 consecutive elements (whole
// float4 loads) per thread.
constexpr int kFrontT = kTile / kW;  // 256
__global__ __launch_bounds__(kFrontT) void k_sq_tot(const float4* __restrict__ x, SqView v) {
  __shared__ double lds[kFrontT / kWave + 1];
  const int t = blockIdx.x;
  const int64_t i0 = (int64_t)t * kTile + (int64_t)threadIdx.x * kW;
  const int b = t * kBlocksPerTile + threadIdx.x;
  float4 q[kW];
#pragma unroll
  for (int j = 0; j < kW; ++j) q[j] = i0 + j < v.n ? x[i0 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = 0; c < v.nch; ++c) {
    double s = 0.0;
    int fl = 0;
    float e[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) {
      e[j] = comp(q[j], c);
      const int f = nf_flags(e[j]);
      fl |= f;
      if (!f) s += (double)e[j];
    }
    float* dst = v.soa + (int64_t)c * v.ns;
    for (int j = 0; j < kW; ++j)
      if (i0 + j < v.n) dst[i0 + j] = e[j];
    if (b < v.nb) v.wflg[(int64_t)c * v.nb + b] = (uint8_t)fl;
    double tot;
    (void)block_scan_excl<kFrontT>(s, lds, &tot);
    if (threadIdx.x == 0) v.ttot[(int64_t)c * v.nk + t] = tot;
  }
}

// ---- 2: boundaries, unmonitored runs, increments ----------------------------------
// One workgroup per (tile, chain); thread = one 16-element window.
__global__ __launch_bounds__(kFrontT) void k_sq_front(SqView v) {
  __shared__ float xs[kTile + kW];
  __shared__ int sbs[kFrontT + 1];
  __shared__ double sA[kFrontT];
  __shared__ double lds[kFrontT / kWave + 1];
  __shared__ double gkey[kKW];
  __shared__ int gid[kKW];
  const int t = blockIdx.x, c = blockIdx.y;
  const int tid = threadIdx.x;
  const int64_t e0 = (int64_t)t * kTile;
  if (t == 0 && c == 0 && tid == 0) *v.err = 0;
  // the tile (and the next tile's first window) of component c
  const float* Xs = v.soa + (int64_t)c * v.ns;
  for (int i = tid; i < kTile + kW; i += kFrontT) xs[i] = e0 + i < v.n ? Xs[e0 + i] : 0.0f;
  // fp64 prefix at the tile start
  const double P = block_sum_global<kFrontT>(v.ttot + (int64_t)c * v.nk, t, lds);
  __syncthreads();
  // the thread's window: fp64 total and prefix
  const int b = t * kBlocksPerTile + tid;
  double wsum = 0.0;
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    const float e = xs[tid * kW + j];
    if (isfinite(e)) wsum += (double)e;
  }
  double ttotal;
  const double wrel = block_scan_excl<kFrontT>(wsum, lds, &ttotal);
  // block start: the element of largest |prefix| in the window (the prefix
  // before the element: the value a block starting there starts from)
  const double wpre = P + wrel;
  double best = wpre, run = wpre;
  int bj = 0;
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    if (j > 0 && fabs(run) > fabs(best) && e0 + tid * kW + j < v.n) {
      best = run;
      bj = j;
    }
    const float e = xs[tid * kW + j];
    if (isfinite(e)) run += (double)e;
  }
  if (b == 0) {
    best = 0.0;
    bj = 0;
  }
  sbs[tid] = tid * kW + bj;  // tile-relative start
  sA[tid] = best;
  if (tid == kFrontT - 1) {
    // the next tile's first block start (same rule), for this tile's last block
    double r2 = P + ttotal, b2 = r2;
    int j2 = 0;
    for (int j = 0; j < kW; ++j) {
      if (j > 0 && fabs(r2) > fabs(b2) && e0 + kTile + j < v.n) {
        b2 = r2;
        j2 = j;
      }
      const float e = xs[kTile + j];
      if (isfinite(e)) r2 += (double)e;
    }
    sbs[kFrontT] = kTile + j2;
  }
  __syncthreads();
  int* bsg = v.bs + (int64_t)c * (v.nb + 1);
  if (b < v.nb) bsg[b] = (int)(e0 + sbs[tid]);
  if (b == v.nb - 1) bsg[v.nb] = (int)v.n;
  // group starts: the block of largest |start value| in each 16-block window
  // (out-of-range blocks never win)
  double key = b < v.nb ? fabs(sA[tid]) : -1.0;
  int kid = b < v.nb ? b : INT_MAX;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    const double ok = __shfl_xor(key, o, 16);
    const int oi = __shfl_xor(kid, o, 16);
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
    for (int i = 0; i < kKW; ++i)
      if (gkey[i] > bk) {
        bk = gkey[i];
        bq = gid[i];
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
    const float G = b == 0 ? 0.0f : (float)sA[tid];
    float s = G;
    double fsum = 0.0;
    for (int i = s0; i < s1; ++i) {
      const float e = xs[i];
      s = s + e;
      if (isfinite(e)) fsum += (double)e;
    }
    incv = isfinite(s) && isfinite(G) ? (double)s - (double)G : fsum;
    v.inc[(int64_t)c * v.nb + b] = incv;
  }
  double itot;
  (void)block_scan_excl<kFrontT>(incv, lds, &itot);
  if (tid == 0) v.tinc[(int64_t)c * v.nk + t] = itot;
}

// ---- 3: leaf, group and superblock maps ------------------------------------------
constexpr int kMapT = 1024;

__device__ __forceinline__ float cand(float G, int e0, int r) {
  return (float)((double)G + ldexp((double)r, e0));
}

__global__ __launch_bounds__(kMapT) void k_sq_maps(SqView v) {
  __shared__ float xs[kMaxSbElems];
  __shared__ Leaf lf[kMaxSbBlocks];
  __shared__ GroupMap gm[kMaxSbGroups];
  __shared__ double Gd[kMaxSbBlocks + 1];
  __shared__ int sbs[kMaxSbBlocks + 1];
  __shared__ int sgs[kMaxSbGroups + 1];
  __shared__ double lds[kMapT / kWave + 1];
  __shared__ int sbad;
  const int k = blockIdx.x, c = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int* bsg = v.bs + (int64_t)c * (v.nb + 1);
  const int* gsg = v.gs + (int64_t)c * (v.ng + 1);
  const int* ksg = v.ks + (int64_t)c * (v.nk + 1);
  // (sizes are checked before each dependent load: a bad table stops the
  // workgroup instead of reading out of range)
  const int ga = ksg[k], gb = ksg[k + 1];
  if (ga < 0 || gb > v.ng || gb - ga < 1 || gb - ga > kMaxSbGroups) {
    if (tid == 0) atomicOr(v.err, 1);
    return;
  }
  const int ba = gsg[ga], bb = gsg[gb];
  if (ba < 0 || bb > v.nb || bb - ba < 1 || bb - ba > kMaxSbBlocks) {
    if (tid == 0) atomicOr(v.err, 1);
    return;
  }
  const int ea = bsg[ba], eb = bsg[bb];
  if (ea < 0 || eb > v.n || eb - ea < 1 || eb - ea > kMaxSbElems) {
    if (tid == 0) atomicOr(v.err, 1);
    return;
  }
  const int ngr = gb - ga, nblk = bb - ba, nel = eb - ea;
  const float* X = v.soa + (int64_t)c * v.ns;
  if (tid == 0) sbad = 0;
  for (int i = tid; i < nel; i += kMapT) xs[i] = X[ea + i];
  for (int i = tid; i <= nblk; i += kMapT) sbs[i] = bsg[ba + i] - ea;
  for (int i = tid; i <= ngr; i += kMapT) sgs[i] = gsg[ga + i] - ba;
  // refined guesses: the fp64 prefix of the blocks' float32 increments
  const double* inc = v.inc + (int64_t)c * v.nb;
  const int tb = ba / kBlocksPerTile;
  double base = block_sum_global<kMapT>(v.tinc + (int64_t)c * v.nk, tb, lds);
  __syncthreads();
  base += block_sum_global<kMapT>(inc + (int64_t)tb * kBlocksPerTile, ba - tb * kBlocksPerTile, lds);
  __syncthreads();
  {
    // nblk <= 511 < kMapT: one increment per thread
    const double iv = tid < nblk ? inc[ba + tid] : 0.0;
    double tot;
    const double pre = block_scan_excl<kMapT>(iv, lds, &tot);
    if (tid < nblk) Gd[tid] = ba + tid == 0 ? 0.0 : base + pre;
  }
  __syncthreads();
  // -- leaves: lane (block, residue pair): runs from candidates rp and rp + 2,
  // interleaved (two independent dependency chains per lane, one round for
  // up to 512 blocks)
  Leaf* leafg = v.leaf + (int64_t)c * v.nb;
  {
    const int bl = tid >> 1, rp = tid & 1;
    const bool act = bl < nblk;
    Run p0, p1;
    float G = 0.0f;
    int e0 = -149;
    if (act) {
      G = candidate_base((float)Gd[bl], kLeafR);
      e0 = grid_exp(G);
      run_init(p0, cand(G, e0, rp));
      run_init(p1, cand(G, e0, rp + 2));
      int s0 = sbs[bl], s1 = sbs[bl + 1];
      if (s0 < 0 || s1 > nel || s1 - s0 < 1 || s1 - s0 > 2 * kW - 1) {
        atomicOr(v.err, 32);
        p0.opaque = true;
        s1 = s0;
      }
      for (int i = s0; i < s1; ++i) {
        const float xv = xs[i];
        run_step(p0, xv, e0);
        run_step(p1, xv, e0);
      }
    } else {
      run_init(p0, 0.0f);
      run_init(p1, 0.0f);
    }
    // the block's lattice: the largest need over its 4 runs
    int need = max(p0.need, p1.need);
    need = max(need, __shfl_xor(need, 1, kWave));
    const bool op0 = __shfl(p0.opaque ? 1 : 0, lane & ~1, kWave) != 0;
    if (act) {
      const int mneed = need == kNoNeed ? 0 : max(0, need - e0);
      const bool exact_only = mneed > kLeafM;
      const int m = exact_only ? 0 : mneed;
      Leaf& o = lf[bl];
      if (rp == 0) {
        o.h.G = G;
        o.h.e0 = e0;
        o.h.m = m;
        o.h.flags = op0 ? kOpaque : 0;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const Run& p = h ? p1 : p0;
        const int r = rp + 2 * h;
        MapEnt en;
        en.E = p.s;
        en.LOu = lo_units((double)p.lo, e0);
        en.HIu = hi_units((double)p.hi, e0);
        if (p.opaque || r >= (1 << m)) {
          en.LOu = 1;
          en.HIu = 0;
        } else if (exact_only) {
          en.LOu = max(en.LOu, 0);
          en.HIu = min(en.HIu, 0);
        }
        o.e[r] = en;
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < nblk * (int)(sizeof(Leaf) / 4); i += kMapT)
    reinterpret_cast<int*>(leafg + ba)[i] = reinterpret_cast<const int*>(lf)[i];
  // -- groups: lane (group, residue), up to 16 residues
  GroupMap* grpg = v.grp + (int64_t)c * v.ng;
  {
    const int gi = tid / kGroupR, r = tid % kGroupR;
    const int c0 = gi < ngr ? sgs[gi] : 0, c1 = gi < ngr ? sgs[gi + 1] : 0;
    const bool gok = c0 >= 0 && c1 > c0 && c1 <= nblk && c1 - c0 <= 2 * kGW - 1;
    if (gi < ngr && !gok) {
      atomicOr(v.err, 2);
      sbad = 1;
    }
    if (gi < ngr && gok) {
      // lattice over the children
      const MapHdr h0 = lf[c0].h;
      int lat = h0.e0 + h0.m;
      for (int j = c0 + 1; j < c1; ++j) {
        const MapHdr hj = lf[j].h;
        if (!(hj.flags & kOpaque)) lat = max(lat, hj.e0 + hj.m);
      }
      int m = max(0, lat - h0.e0);
      const bool exact_only = m > kGroupM;
      if (exact_only) m = 0;
      const int R = 1 << m;
      const float G = candidate_base(h0.G, R);
      const int e0 = grid_exp(G);
      GroupMap& o = gm[gi];
      if (r == 0) {
        o.h.G = G;
        o.h.e0 = e0;
        o.h.m = m;
        o.h.flags = 0;
      }
      MapEnt en;
      en.E = 0.0f;
      en.LOu = 1;
      en.HIu = 0;
      if (r < R) {
        float x = cand(G, e0, r);
        double clo = -INFINITY, chi = INFINITY;
        bool ok = true;
        for (int j = c0; j < c1 && ok; ++j) ok = through(x, clo, chi, lf[j].h, lf[j].e);
        if (ok) {
          if (exact_only) {
            clo = fmax(clo, 0.0);
            chi = fmin(chi, 0.0);
          }
          en.E = x;
          en.LOu = lo_units(clo, e0);
          en.HIu = hi_units(chi, e0);
        }
      }
      o.e[r] = en;
    }
  }
  __syncthreads();
  for (int i = tid; i < ngr * (int)(sizeof(GroupMap) / 4); i += kMapT)
    reinterpret_cast<int*>(grpg + ga)[i] = reinterpret_cast<const int*>(gm)[i];
  // -- the superblock: lanes = residues, up to 64
  if (tid < kWave && sbad) {
    SbMap* o = v.sbm + (int64_t)c * v.nk + k;
    if (tid == 0) o->h.flags = kOpaque;
  } else if (tid < kWave) {
    const int r = tid;
    const MapHdr h0 = gm[0].h;
    int lat = h0.e0 + h0.m;
    for (int j = 1; j < ngr; ++j) lat = max(lat, gm[j].h.e0 + gm[j].h.m);
    int m = max(0, lat - h0.e0);
    const bool exact_only = m > kSbM;
    if (exact_only) m = 0;
    const int R = 1 << m;
    const float G = candidate_base(h0.G, R);
    const int e0 = grid_exp(G);
    SbMap* o = v.sbm + (int64_t)c * v.nk + k;
    if (r == 0) {
      MapHdr h;
      h.G = G;
      h.e0 = e0;
      h.m = m;
      h.flags = 0;
      o->h = h;
    }
    MapEnt en;
    en.E = 0.0f;
    en.LOu = 1;
    en.HIu = 0;
    if (r < R) {
      float x = cand(G, e0, r);
      double clo = -INFINITY, chi = INFINITY;
      bool ok = true;
      for (int j = 0; j < ngr && ok; ++j) ok = through(x, clo, chi, gm[j].h, gm[j].e);
      if (ok) {
        if (exact_only) {
          clo = fmax(clo, 0.0);
          chi = fmin(chi, 0.0);
        }
        en.E = x;
        en.LOu = lo_units(clo, e0);
        en.HIu = hi_units(chi, e0);
      }
    }
    o->e[r] = en;
  }
}

// ---- 4: the walk -------------------------------------------------------------------
// One wavefront per chain.  Superblock maps are staged into LDS in chunks of
// kWalkC (the next chunk's loads in flight while the current one is
// walked); a failed superblock check loads that superblock's group maps,
// a failed group check the group's leaves, a failed leaf check the block's
// elements -- the reference's own adds.
constexpr int kWalkC = 16;
constexpr int kSbF4 = sizeof(SbMap) / 16;  // 64 float4 per superblock map

struct WalkLds {
  SbMap sb[2][kWalkC];
  GroupMap g[kMaxSbGroups];
  Leaf l[2 * kGW];
  float x[2 * kW];
  int gs[kMaxSbGroups + 1];
  int bs[2 * kGW + 1];
};

// map (header h, entries e[]) applied to the exact s (all lanes agree)
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

__global__ __launch_bounds__(kWave) void k_sq_walk(SqView v, float* __restrict__ out) {
  __shared__ WalkLds W;
  const int c = blockIdx.x, lane = threadIdx.x;
  const SbMap* sbm = v.sbm + (int64_t)c * v.nk;
  const GroupMap* grp = v.grp + (int64_t)c * v.ng;
  const Leaf* leaf = v.leaf + (int64_t)c * v.nb;
  const int* bsg = v.bs + (int64_t)c * (v.nb + 1);
  const int* gsg = v.gs + (int64_t)c * (v.ng + 1);
  const int* ksg = v.ks + (int64_t)c * (v.nk + 1);
  const float* X = v.soa + (int64_t)c * v.ns;
  int* st = v.stats ? v.stats + c * 8 : nullptr;
  const uint64_t t0 = st ? __builtin_amdgcn_s_memtime() : 0;
  int n_sb = 0, n_sbh = 0, n_g = 0, n_gh = 0, n_l = 0, n_lh = 0, n_ser = 0;
  float s = 0.0f;
  int64_t pos_nf = -1;  // element index where s became non-finite
  // chunk staging: lane copies float4 lane + 64 j of the chunk
  float4 pre[kWalkC];
  auto issue = [&](int ch) {
    const float4* src = reinterpret_cast<const float4*>(sbm + (int64_t)ch * kWalkC);
    const int cnt = min(kWalkC, v.nk - ch * kWalkC) * kSbF4;
#pragma unroll
    for (int j = 0; j < kWalkC; ++j) {
      const int i = lane + j * kWave;
      pre[j] = i < cnt ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto land = [&](int buf) {
    float4* dst = reinterpret_cast<float4*>(&W.sb[buf][0]);
#pragma unroll
    for (int j = 0; j < kWalkC; ++j) dst[lane + j * kWave] = pre[j];
  };
  const int nchunk = (v.nk + kWalkC - 1) / kWalkC;
  if (nchunk > 0) {
    issue(0);
    land(0);
  }
  __syncthreads();
  for (int ch = 0; ch < nchunk && pos_nf < 0; ++ch) {
    if (ch + 1 < nchunk) issue(ch + 1);
    const int kend = min(v.nk, (ch + 1) * kWalkC);
    for (int k = ch * kWalkC; k < kend && pos_nf < 0; ++k) {
      const SbMap& M = W.sb[ch & 1][k - ch * kWalkC];
      ++n_sb;
      if (walk_try(s, M.h, M.e, kSbM)) {
        ++n_sbh;
        continue;
      }
      // descend: the superblock's groups
      const int ga = ksg[k], gb = ksg[k + 1];
      const int ngr = gb - ga;
      if (ngr < 1 || ngr > kMaxSbGroups || ga < 0 || gb > v.ng) {
        if (lane == 0) atomicOr(v.err, 4);
        pos_nf = v.n;
        s = __int_as_float(0x7fc00000);
        break;
      }
      {
        const int4* src = reinterpret_cast<const int4*>(grp + ga);
        int4* dst = reinterpret_cast<int4*>(W.g);
        for (int i = lane; i < ngr * (int)(sizeof(GroupMap) / 16); i += kWave) dst[i] = src[i];
        for (int i = lane; i <= ngr; i += kWave) W.gs[i] = gsg[ga + i];
      }
      __syncthreads();
      for (int q = 0; q < ngr && pos_nf < 0; ++q) {
        ++n_g;
        if (walk_try(s, W.g[q].h, W.g[q].e, kGroupM)) {
          ++n_gh;
          continue;
        }
        const int b0 = W.gs[q], b1 = W.gs[q + 1];
        if (b1 - b0 < 1 || b1 - b0 > 2 * kGW - 1 || b0 < 0 || b1 > v.nb) {
          if (lane == 0) atomicOr(v.err, 8);
          pos_nf = v.n;
          s = __int_as_float(0x7fc00000);
          break;
        }
        __syncthreads();
        {
          const int4* src = reinterpret_cast<const int4*>(leaf + b0);
          int4* dst = reinterpret_cast<int4*>(W.l);
          for (int i = lane; i < (b1 - b0) * (int)(sizeof(Leaf) / 16); i += kWave) dst[i] = src[i];
          for (int i = lane; i <= b1 - b0; i += kWave) W.bs[i] = bsg[b0 + i];
        }
        __syncthreads();
        for (int bl = 0; bl < b1 - b0; ++bl) {
          ++n_l;
          if (walk_try(s, W.l[bl].h, W.l[bl].e, kLeafM)) {
            ++n_lh;
            continue;
          }
          // the block by the reference's own adds
          ++n_ser;
          const int e0 = W.bs[bl], e1 = W.bs[bl + 1];
          if (e1 - e0 < 1 || e1 - e0 > 2 * kW - 1 || e0 < 0 || e1 > v.n) {
            if (lane == 0) atomicOr(v.err, 16);
            pos_nf = v.n;
            s = __int_as_float(0x7fc00000);
            break;
          }
          __syncthreads();
          if (lane < e1 - e0) W.x[lane] = X[e0 + lane];
          __syncthreads();
          for (int i = 0; i < e1 - e0; ++i) s = s + W.x[i];
          if (!isfinite(s)) {
            pos_nf = e1;
            break;
          }
        }
        __syncthreads();
      }
      __syncthreads();
    }
    if (ch + 1 < nchunk) land((ch + 1) & 1);
    __syncthreads();
  }
  if (pos_nf >= 0) {
    // inf / NaN absorbs every finite element: only NaN or an opposite
    // infinity later can still change it.  Serial to the next window, then
    // the window flags.
    int64_t i = pos_nf;
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
    if (c == 0 && v.stats) v.stats[32] = *v.err;
    if (st) {
      st[0] = n_sb;
      st[1] = n_sbh;
      st[2] = n_g;
      st[3] = n_gh;
      st[4] = n_l;
      st[5] = n_lh;
      st[6] = n_ser;
      st[7] = (int)min<uint64_t>(INT_MAX, __builtin_amdgcn_s_memtime() - t0);
    }
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
  v.soa = (float*)take(sizeof(float) * nch * (size_t)v.ns);
  v.wflg = (uint8_t*)take((size_t)nch * v.nb);
  v.err = (int*)take(sizeof(int));
  v.ttot = (double*)take(sizeof(double) * nch * (size_t)v.nk);
  v.bs = (int*)take(sizeof(int) * nch * (size_t)(v.nb + 1));
  v.gs = (int*)take(sizeof(int) * nch * (size_t)(v.ng + 1));
  v.ks = (int*)take(sizeof(int) * nch * (size_t)(v.nk + 1));
  v.inc = (double*)take(sizeof(double) * nch * (size_t)v.nb);
  v.tinc = (double*)take(sizeof(double) * nch * (size_t)v.nk);
  v.leaf = (Leaf*)take(sizeof(Leaf) * nch * (size_t)v.nb);
  v.grp = (GroupMap*)take(sizeof(GroupMap) * nch * (size_t)v.ng);
  v.sbm = (SbMap*)take(sizeof(SbMap) * nch * (size_t)v.nk);
  return off;
}

size_t seqsum_bytes(int64_t n) {
  SqView v;
  return sq_layout(v, std::max<int64_t>(n, 1), 4, nullptr);
}

// out[c] for c < nch: the sequential float sum of component c of x[0..n).
// stages (debug): bit 0 the front kernel, bit 1 the maps, bit 2 the walk.
int seqsum_enqueue(const float4* d_x, int64_t n, int nch, void* ws, float* d_out, hipStream_t st,
                   int* d_stats, int stages) {
  if (nch < 1 || nch > 4 || n < 0) return RST_E_ARG;
  if (n == 0) {
    RST_HIP(hipMemsetAsync(d_out, 0, sizeof(float) * nch, st));
    return RST_OK;
  }
  if (n > (int64_t)INT_MAX - 2 * kTile) return RST_E_ARG;
  SqView v;
  sq_layout(v, n, nch, (char*)ws);
  v.stats = d_stats;
  if (stages & 1) {
    k_sq_tot<<<v.nk, kFrontT, 0, st>>>(d_x, v);
    k_sq_front<<<dim3(v.nk, nch), kFrontT, 0, st>>>(v);
  }
  if (stages & 2) k_sq_maps<<<dim3(v.nk, nch), kMapT, 0, st>>>(v);
  if (stages & 4) k_sq_walk<<<nch, kWave, 0, st>>>(v, d_out);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

}  // namespace rst
