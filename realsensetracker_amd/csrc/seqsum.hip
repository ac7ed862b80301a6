// seqsum.hip -- the reference's sequential float32 sums, computed in parallel
// and bit-exact.
//
// RST_SUM_REF replays `dst_mean += dst.GetPoint(j)` / `cost += dist_sqr`
// (align_icp.cpp:113,120) and ComputeCentroid's loop
// (point_cloud_utils.cpp:94-96): s_{k+1} = fl(s_k + x_k) in float32,
// round-to-nearest-even, k ascending from s_0 = +0.  A dependent chain of n
// adds (k_seq_sum4 in icp.hip, ~1.4 ms at 300k points) -- this file gets the
// same bits with almost all of the chain taken in jumps.
//
// Why a jump is exact.  While every exact intermediate y_k = s_k + x_k lies
// in one binade [2^e, 2^(e+1)] (or its negative), fl() rounds to the fixed
// grid g = 2^(e-23), and s_k itself is a multiple of g.  With S = s / g an
// integer in [2^23, 2^24]:
//     S_{k+1} = S_k + a_k + r_k,   a_k = floor(x_k / g),
// r_k = 1 if frac(x_k / g) > 1/2, 0 if < 1/2, and on an exact tie the choice
// that makes S_{k+1} even (ties-to-even on the mantissa = on S).  So an
// element is a map S -> S + d[S & 1], and maps of that form (two offsets,
// indexed by the parity of the input) are closed under composition:
//     (f then g).d[p] = f.d[p] + g.d[(p + f.d[p]) & 1].
// A run of elements under binade e is therefore six integers: d[2] and the
// lowest / highest exact intermediate y/g relative to the start, lo[2] /
// hi[2] (floor / ceil bounds).  Given the actual start S, the run is valid
// iff S + lo[p] >= 2^23 and S + hi[p] <= 2^24 (negative sums: -2^24 and
// -2^23) -- then every step rounded on grid g, and s_end = (S + d[p]) g
// exactly.  Validity is checked at run time against the true S; a run that
// fails is never used, so the result never depends on a guess.
//
// Kernels (per chain c = one float component of the float4 stream):
//   k_sq_tot    per block of 64 elements: fp64 total, non-finite flags;
//   k_sq_scan   exclusive fp64 prefix of the totals (an APPROXIMATE start
//               value per block: it only picks which binades to tabulate);
//   k_sq_blocks per block: the run maps for the 3 binades around the
//               approximate start (e-1, e, e+1), slot e mod 3, and a
//               `problem` hint when the approximate path crosses a binade;
//   k_sq_super  per 64 blocks: the composed maps for 3 binades;
//   k_sq_walk   one wavefront per chain walks the stream with the true s:
//               64 superblock maps at a time (wave prefix-composition,
//               first invalid lane stops the jump), else 64 block maps,
//               else one block serially (the reference's own adds).
// On a real 640x480 frame the x chain (the one that crosses zero) walks 255
// blocks serially out of 4688; y and z fewer than 30.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>

#include "rst_device.hpp"
#include "rst_internal.hpp"

namespace rst {
namespace {

constexpr int kSqB = 64;          // elements per block (one wavefront)
constexpr int kSqS = 64;          // blocks per superblock
constexpr int kInv = 1 << 28;     // invalid / identity bounds
constexpr int kLim = 1 << 25;     // beyond this a map can never be valid
constexpr int kEmin = -125, kEmax = 126;  // binades with normal, finite grids
constexpr int kNoE = INT_MIN;

// one run map; the record layout in memory is two int4: {e, d0, d1, lo0},
// {lo1, hi0, hi1, problem}.  Scalar members and selects only: an array
// indexed by the run-time parity would live in scratch, and a scratch load
// waits for every global load in flight (the walker's prefetch).
struct Fn {
  int d0, d1, lo0, lo1, hi0, hi1;
  __device__ __forceinline__ int d(int p) const { return p ? d1 : d0; }
  __device__ __forceinline__ int lo(int p) const { return p ? lo1 : lo0; }
  __device__ __forceinline__ int hi(int p) const { return p ? hi1 : hi0; }
};

__device__ __forceinline__ Fn fn_make(int d0, int d1, int lo0, int lo1, int hi0, int hi1) {
  Fn f;
  f.d0 = d0;
  f.d1 = d1;
  f.lo0 = lo0;
  f.lo1 = lo1;
  f.hi0 = hi0;
  f.hi1 = hi1;
  return f;
}
__device__ __forceinline__ Fn fn_ident() { return fn_make(0, 0, kInv, kInv, -kInv, -kInv); }
__device__ __forceinline__ Fn fn_invalid() { return fn_make(0, 0, -kInv, -kInv, kInv, kInv); }

// one parity of f then g
__device__ __forceinline__ void fn_compose1(int fd, int flo, int fhi, const Fn& g, int p, int& d,
                                            int& lo, int& hi) {
  const int q = (p + fd) & 1;
  d = fd + g.d(q);
  lo = min(flo, fd + g.lo(q));
  hi = max(fhi, fd + g.hi(q));
  if (lo < -kLim || hi > kLim || d > kLim || d < -kLim) {  // saturate: never valid
    d = 0;
    lo = -kInv;
    hi = kInv;
  }
}
// f then g
__device__ __forceinline__ Fn fn_compose(const Fn& f, const Fn& g) {
  Fn h;
  fn_compose1(f.d0, f.lo0, f.hi0, g, 0, h.d0, h.lo0, h.hi0);
  fn_compose1(f.d1, f.lo1, f.hi1, g, 1, h.d1, h.lo1, h.hi1);
  return h;
}

// the map of one element x under binade e (grid 2^(e-23))
__device__ __forceinline__ Fn fn_elem(float x, int e) {
  if (!isfinite(x)) return fn_invalid();
  const double X = ldexp((double)x, 23 - e);
  if (!(fabs(X) < (double)kLim)) return fn_invalid();
  const double fa = floor(X);
  const double fr = X - fa;  // exact
  const int a = (int)fa;
  const int hi = a + (fr > 0.0 ? 1 : 0);
  if (fr == 0.5)  // tie: the even result
    return fn_make(a + ((0 + a) & 1), a + ((1 + a) & 1), a, a, hi, hi);
  const int d = a + (fr > 0.5 ? 1 : 0);
  return fn_make(d, d, a, a, hi, hi);
}

// DPP moves (VALU lane shifts, no LDS round trip): row_shr:k within rows of
// 16 lanes, then row_bcast:15 / row_bcast:31 across rows; lanes without a
// source (or outside row_mask) get `old` = the identity map.
template <int Ctrl, int RowMask>
__device__ __forceinline__ Fn fn_dpp(const Fn& f) {
  const Fn id = fn_ident();
  return fn_make(__builtin_amdgcn_update_dpp(id.d0, f.d0, Ctrl, RowMask, 0xf, false),
                 __builtin_amdgcn_update_dpp(id.d1, f.d1, Ctrl, RowMask, 0xf, false),
                 __builtin_amdgcn_update_dpp(id.lo0, f.lo0, Ctrl, RowMask, 0xf, false),
                 __builtin_amdgcn_update_dpp(id.lo1, f.lo1, Ctrl, RowMask, 0xf, false),
                 __builtin_amdgcn_update_dpp(id.hi0, f.hi0, Ctrl, RowMask, 0xf, false),
                 __builtin_amdgcn_update_dpp(id.hi1, f.hi1, Ctrl, RowMask, 0xf, false));
}
// inclusive ordered prefix: lane j gets map_0 then ... then map_j
// (compose(ident, f) == f, so identity fills are exact)
__device__ __forceinline__ Fn fn_wave_scan(Fn f, int lane) {
  (void)lane;
  f = fn_compose(fn_dpp<0x111, 0xf>(f), f);  // row_shr:1
  f = fn_compose(fn_dpp<0x112, 0xf>(f), f);  // row_shr:2
  f = fn_compose(fn_dpp<0x114, 0xf>(f), f);  // row_shr:4
  f = fn_compose(fn_dpp<0x118, 0xf>(f), f);  // row_shr:8
  f = fn_compose(fn_dpp<0x142, 0xa>(f), f);  // row_bcast:15 -> rows 1, 3
  f = fn_compose(fn_dpp<0x143, 0xc>(f), f);  // row_bcast:31 -> rows 2, 3
  return f;
}
// ordered composition of the wave's 64 maps, in every lane's... lane 63
__device__ __forceinline__ Fn fn_wave_total(Fn f, int lane) {
  f = fn_wave_scan(f, lane);
  return fn_make(__shfl(f.d0, kWave - 1, kWave), __shfl(f.d1, kWave - 1, kWave),
                 __shfl(f.lo0, kWave - 1, kWave), __shfl(f.lo1, kWave - 1, kWave),
                 __shfl(f.hi0, kWave - 1, kWave), __shfl(f.hi1, kWave - 1, kWave));
}

__device__ __forceinline__ int slot_of(int e) { return ((e % 3) + 3) % 3; }

__device__ __forceinline__ void rec_store(int4* rec, int e, const Fn& f, int problem) {
  rec[0] = make_int4(e, f.d0, f.d1, f.lo0);
  rec[1] = make_int4(f.lo1, f.hi0, f.hi1, problem);
}
__device__ __forceinline__ Fn rec_fn(int4 a, int4 b) { return fn_make(a.y, a.z, a.w, b.x, b.y, b.z); }

// binade of a float: e with 2^e <= |s| < 2^(e+1), kNoE outside the normal range
__device__ __forceinline__ int binade_f(float s) {
  const uint32_t ex = (__float_as_uint(s) >> 23) & 0xffu;
  const int e = (int)ex - 127;
  return (e >= kEmin && e <= kEmax) ? e : kNoE;
}
__device__ __forceinline__ int binade_d(double a) {
  if (!(fabs(a) >= 0x1p-125 && fabs(a) < 0x1p127)) return kNoE;
  const int e = ilogb(a);
  return (e >= kEmin && e <= kEmax) ? e : kNoE;
}

__device__ __forceinline__ float comp(const float4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}

// non-finite flags of a value: 1 NaN, 2 +inf, 4 -inf (block flags: 8 all zero)
__device__ __forceinline__ int nf_flags(float x) {
  if (isnan(x)) return 1;
  if (isinf(x)) return x > 0 ? 2 : 4;
  return 0;
}

struct SqView {
  int64_t n;
  int nb, nsb, nch;
  double* tot;   // [nch][nb]
  double* pre;   // [nch][nb]
  int* flg;      // [nch][nb]
  int4* brec;    // [nch][3][nb][2]
  int4* srec;    // [nch][3][nsb][2]
  int* sflg;     // [nch][nsb]
  float* soa;    // [nch][nb * 64] each component contiguous, zero-padded (the walker's DMA source)
  int* stats;    // optional, per chain 8 ints: l2 tries / jumps, l1 tries / jumps, serial, zero skips, steps
};

// ---- 1: block totals (fp64) and non-finite flags ------------------------------------
__global__ __launch_bounds__(256) void k_sq_tot(const float4* __restrict__ x, SqView v) {
  const int lane = threadIdx.x & (kWave - 1);
  const int b = blockIdx.x * 4 + threadIdx.x / kWave;
  if (b >= v.nb) return;
  const int64_t i = (int64_t)b * kSqB + lane;
  const float4 q = i < v.n ? x[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = 0; c < v.nch; ++c) {
    const float xc = comp(q, c);
    v.soa[(int64_t)c * v.nb * kSqB + i] = xc;
    const int fl = nf_flags(xc);
    const double s = wave_sum(fl ? 0.0 : (double)xc);
    const int f = (__ballot(fl & 1) ? 1 : 0) | (__ballot(fl & 2) ? 2 : 0) | (__ballot(fl & 4) ? 4 : 0) |
                  (__ballot(xc != 0.0f) ? 0 : 8);  // 8: every element is +-0
    if (lane == 0) {
      v.tot[(int64_t)c * v.nb + b] = s;
      v.flg[(int64_t)c * v.nb + b] = f;
    }
  }
}

// ---- 2: exclusive prefix of the block totals (one workgroup) ----------------------------
constexpr int kScanT = 1024;
__global__ __launch_bounds__(kScanT) void k_sq_scan(SqView v) {
  __shared__ double wtot[kScanT / kWave];
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const int per = (v.nb + kScanT - 1) / kScanT;
  const int b0 = t * per, b1 = min(v.nb, b0 + per);
  for (int c = 0; c < v.nch; ++c) {
    const double* tot = v.tot + (int64_t)c * v.nb;
    double* pre = v.pre + (int64_t)c * v.nb;
    double s = 0.0;
    for (int b = b0; b < b1; ++b) s += tot[b];
    // inclusive wave scan, then the wave totals
    double inc = s;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const double y = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += y;
    }
    if (lane == kWave - 1) wtot[w] = inc;
    __syncthreads();
    if (w == 0) {
      double a = lane < kScanT / kWave ? wtot[lane] : 0.0;
      double ia = a;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const double y = __shfl_up(ia, o, kWave);
        if (lane >= o) ia += y;
      }
      if (lane < kScanT / kWave) wtot[lane] = ia - a;
    }
    __syncthreads();
    double acc = wtot[w] + inc - s;
    for (int b = b0; b < b1; ++b) {
      pre[b] = acc;
      acc += tot[b];
    }
    __syncthreads();  // wtot is rewritten by the next chain
  }
}

// ---- 3: per-block run maps for 3 binades ------------------------------------------------
__global__ __launch_bounds__(256) void k_sq_blocks(const float4* __restrict__ x, SqView v) {
  const int lane = threadIdx.x & (kWave - 1);
  const int b = blockIdx.x * 4 + threadIdx.x / kWave;
  if (b >= v.nb) return;
  const int64_t i = (int64_t)b * kSqB + lane;
  const bool in = i < v.n;
  const float4 q = in ? x[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = 0; c < v.nch; ++c) {
    const float xc = comp(q, c);
    const double a0 = v.pre[(int64_t)c * v.nb + b];
    // the approximate path through the block (inclusive prefix, fp64)
    double inc = in && isfinite(xc) ? (double)xc : 0.0;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const double y = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += y;
    }
    const double ak = a0 + inc;
    int eb = binade_d(a0);
    if (eb == kNoE) eb = binade_d(__shfl(ak, kWave - 1, kWave));
    // hint: the approximate path leaves eb's binade or comes near its edges
    bool prob = eb == kNoE || (in && !isfinite(xc));
    if (in && eb != kNoE) {
      const double m = fabs(ak) * exp2(-(double)eb);  // in [1, 2) when inside
      prob = prob || !(m >= 1.0 + 0x1p-10 && m <= 2.0 - 0x1p-10);
    }
    const int problem = __ballot(prob) ? 1 : 0;
    int4* rec = v.brec + ((int64_t)c * 3) * v.nb * 2;
#pragma unroll
    for (int k = -1; k <= 1; ++k) {
      const int e = eb == kNoE ? kNoE : eb + k;
      const bool ev = e != kNoE && e >= kEmin && e <= kEmax;
      Fn f = !in ? fn_ident() : (ev ? fn_elem(xc, e) : fn_invalid());
      f = fn_wave_total(f, lane);
      if (lane == 0) {
        const int sl = eb == kNoE ? k + 1 : slot_of(eb + k);  // 3 distinct slots
        rec_store(rec + ((int64_t)sl * v.nb + b) * 2, ev ? e : kNoE, f, problem);
      }
    }
  }
}

// ---- 4: superblock maps (64 blocks composed) --------------------------------------------
__global__ __launch_bounds__(256) void k_sq_super(SqView v) {
  const int lane = threadIdx.x & (kWave - 1);
  const int sb = blockIdx.x * 4 + threadIdx.x / kWave;
  if (sb >= v.nsb) return;
  const int b = sb * kSqS + lane;
  const bool in = b < v.nb;
  for (int c = 0; c < v.nch; ++c) {
    const int4* brec = v.brec + ((int64_t)c * 3) * v.nb * 2;
    int4* srec = v.srec + ((int64_t)c * 3) * v.nsb * 2;
    const int fl = in ? v.flg[(int64_t)c * v.nb + b] : 0;
    int orf = fl;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) orf |= __shfl_xor(orf, o, kWave);
    // candidate binades: the first block's three slots
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int e = brec[((int64_t)s * v.nb + sb * kSqS) * 2].x;
      Fn f;
      if (!in) {
        f = fn_ident();
      } else if (e == kNoE) {
        f = fn_invalid();
      } else {
        const int4* r = brec + ((int64_t)slot_of(e) * v.nb + b) * 2;
        const int4 r0 = r[0], r1 = r[1];
        f = r0.x == e ? rec_fn(r0, r1) : fn_invalid();
      }
      f = fn_wave_total(f, lane);
      if (lane == 0) rec_store(srec + ((int64_t)s * v.nsb + sb) * 2, e, f, 0);
    }
    if (lane == 0) v.sflg[(int64_t)c * v.nsb + sb] = orf;
  }
}

// ---- 5: the walk (one wavefront per chain) ----------------------------------------------
// Jump over the leading units whose maps (lane j: f, usable_j) are valid
// from the true s under binade e; returns the units jumped (0: none).
__device__ __forceinline__ int jump_scan(Fn f, bool usable, int e, float& s, int lane) {
  const uint64_t bad = __ballot(!usable);
  const int first_bad = bad ? __builtin_ctzll(bad) : kWave;
  if (first_bad == 0) return 0;
  if (!usable) f = fn_invalid();
  f = fn_wave_scan(f, lane);
  const uint32_t bits = __float_as_uint(s);
  const int S0 = (int)((bits & 0x7fffffu) | 0x800000u);
  const int S = (bits >> 31) ? -S0 : S0;
  const int p = S & 1;
  const int dd = f.d(p), lo = f.lo(p), hi = f.hi(p);
  bool val = lane < first_bad;
  if (S > 0)
    val = val && S + lo >= (1 << 23) && S + hi <= (1 << 24);
  else
    val = val && S + lo >= -(1 << 24) && S + hi <= -(1 << 23);
  const uint64_t vm = __ballot(val);
  const int k = (~vm) ? __builtin_ctzll(~vm) : kWave;  // leading valid lanes
  if (k == 0) return 0;
  const int Sd = __shfl(dd, k - 1, kWave);
  s = ldexpf((float)(S + Sd), e - 23);
  return k;
}

// The walker works one superblock (64 blocks = 4096 elements) at a time out
// of LDS: the component's elements, the blocks' 3-slot records and flags
// (superblock records are read from global memory on the rare aligned
// attempts).  The next superblock streams into the other LDS buffer by
// direct global->LDS loads (global_load_lds: no registers, so nothing in the
// walk waits for them) while the current one is walked; the only wait is
// at the superblock boundary.
struct SbBuf {
  float d[kSqS * kSqB];   // element k * 64 + j of the superblock
  int4 r0[3][kSqS];       // block j's records (first half)
  int4 r1[3][kSqS];       //                    (second half)
  int flg[kSqS];
};

// global -> LDS DMA as inline asm (the guide's recipe: M0 = the wave-uniform
// LDS base, written and restored in the same statement).  hipcc does not
// see these loads, so it inserts no wait before the walker's LDS reads of
// the CURRENT buffer (with the builtin it drains the prefetch at every
// read); their completion is awaited explicitly (wait_vm0) at the
// superblock boundary, before the buffer they fill is read.
__device__ __forceinline__ uint32_t lds_addr(const void* l) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)l;
}
__device__ __forceinline__ void glds4(const void* g, void* l) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_addr(l)))
               : "memory");
}
__device__ __forceinline__ void glds16(const void* g, void* l) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_addr(l)))
               : "memory");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// issue superblock sb's loads into B: 16 + 1 + 6 = kSbDma DMA instructions
// (clamped indices: every lane loads)
constexpr int kSbDma = 23;
__device__ __forceinline__ void sb_issue(const SqView& v, int c, int sb, int lane, SbBuf& B) {
  const int base = sb * kSqS;
  const float* xs = v.soa + (int64_t)c * v.nb * kSqB + (int64_t)base * kSqB;  // padded to nb * 64
  const int nblk = min(kSqS, v.nb - base);
#pragma unroll
  for (int k = 0; k < kSqS / 4; ++k) {  // 4 blocks (1 KiB) per instruction
    const int blk4 = min(4 * k + lane / 16, nblk - 1);
    glds16(xs + (int64_t)blk4 * kSqB + (lane % 16) * 4, &B.d[k * 4 * kSqB]);
  }
  const int blk = min(base + lane, v.nb - 1);
  glds4(v.flg + (int64_t)c * v.nb + blk, &B.flg[0]);
#pragma unroll
  for (int sl = 0; sl < 3; ++sl) {
    const int4* r = v.brec + (((int64_t)c * 3 + sl) * v.nb + blk) * 2;
    glds16(r, &B.r0[sl][0]);
    glds16(r + 1, &B.r1[sl][0]);
  }
}
// wait until at most `batches` superblock issues are still in flight
__device__ __forceinline__ void wait_batches(int batches) {
  if (batches >= 2)
    asm volatile("s_waitcnt vmcnt(46)" ::: "memory");
  else if (batches == 1)
    asm volatile("s_waitcnt vmcnt(23)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

constexpr int kSbBufs = 3;  // the current superblock + two in flight
__global__ __launch_bounds__(kWave) void k_sq_walk(const float4* __restrict__ x, SqView v,
                                                   float* __restrict__ out) {
  (void)x;
  __shared__ SbBuf Bs[kSbBufs];
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  float s = 0.0f;
  int b = 0, cur = -1;
  int lo_iss = 0, hi_iss = -1;  // superblocks [lo_iss, hi_iss] issued, possibly in flight
  const uint64_t tw = v.stats ? __builtin_amdgcn_s_memtime() : 0;
  while (b < v.nb) {
    const int sb = b / kSqS, bo = b % kSqS;
    if (sb != cur) {
      if (sb < lo_iss || sb > hi_iss) {  // not prefetched (start, or a long jump)
        wait_vm0();
        sb_issue(v, c, sb, lane, Bs[sb % kSbBufs]);
        lo_iss = hi_iss = sb;
      }
      wait_batches(hi_iss - sb);
      cur = sb;
      lo_iss = sb;
      while (hi_iss < sb + kSbBufs - 1 && hi_iss + 1 < v.nsb) {
        ++hi_iss;
        sb_issue(v, c, hi_iss, lane, Bs[hi_iss % kSbBufs]);
      }
    }
    SbBuf& B = Bs[cur % kSbBufs];
    if (!isfinite(s)) {
      // inf / NaN absorbs every finite element: only NaN or an opposite
      // infinity in the rest can still change it
      wait_vm0();
      int orf = 0;
      for (int j = b + lane; j < v.nb; j += kWave) orf |= v.flg[(int64_t)c * v.nb + j];
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) orf |= __shfl_xor(orf, o, kWave);
      if ((orf & 1) || (s > 0 && (orf & 4)) || (s < 0 && (orf & 2))) s = __int_as_float(0x7fc00000);
      break;
    }
    const int e = binade_f(s);
    if (e != kNoE) {
      const int sl = slot_of(e);
      if (bo == 0) {  // superblocks sb, sb + 1, ... (global loads: rare)
        int4 r0 = make_int4(kNoE, 0, 0, 0), r1 = make_int4(0, 0, 0, 1);
        if (sb + lane < v.nsb) {
          const int4* q = v.srec + (((int64_t)c * 3 + sl) * v.nsb + sb + lane) * 2;
          r0 = q[0];
          r1 = q[1];
        }
        const bool ok = r0.x == e;
        const int k = jump_scan(ok ? rec_fn(r0, r1) : fn_invalid(), ok, e, s, lane);
        if (v.stats && lane == 0) {
          v.stats[c * 8 + 0]++;
          v.stats[c * 8 + 1] += k > 0;
        }
        if (k > 0) {
          b = min(v.nb, b + k * kSqS);
          continue;
        }
      }
      // blocks, up to the superblock's end
      if (!B.r1[sl][bo].w) {  // the first block is not a hinted crossing
        const int j = bo + lane;
        int4 r0 = make_int4(kNoE, 0, 0, 0), r1 = make_int4(0, 0, 0, 1);
        if (j < kSqS && b + lane < v.nb) {
          r0 = B.r0[sl][j];
          r1 = B.r1[sl][j];
        }
        const bool ok = r0.x == e && !(r1.w && lane > 0);
        const int k = jump_scan(ok ? rec_fn(r0, r1) : fn_invalid(), ok, e, s, lane);
        if (v.stats && lane == 0) {
          v.stats[c * 8 + 2]++;
          v.stats[c * 8 + 3] += k > 0;
        }
        if (k > 0) {
          b += k;
          continue;
        }
      }
    } else if (s == 0.0f && (B.flg[bo] & 8)) {  // +0 plus a block of zeros
      if (v.stats && lane == 0) v.stats[c * 8 + 5]++;
      ++b;
      continue;
    }
    // one block in the reference's order
    const int m = (int)min<int64_t>(kSqB, v.n - (int64_t)b * kSqB);
    if (v.stats && lane == 0) v.stats[c * 8 + 4]++;
    const uint64_t t0 = v.stats ? __builtin_amdgcn_s_memtime() : 0;
    if (lane == 0) {
      const float* d = B.d + bo * kSqB;
      if (m == kSqB) {
        const float4* q4 = reinterpret_cast<const float4*>(d);
#pragma unroll 4
        for (int t = 0; t < kSqB / 4; ++t) {
          const float4 q = q4[t];
          s = s + q.x;
          s = s + q.y;
          s = s + q.z;
          s = s + q.w;
        }
      } else {
        for (int t = 0; t < m; ++t) s = s + d[t];
      }
    }
    s = __shfl(s, 0, kWave);
    if (v.stats && lane == 0) v.stats[c * 8 + 6] += (int)(__builtin_amdgcn_s_memtime() - t0);
    ++b;
  }
  wait_vm0();  // no load in flight at exit
  if (v.stats && lane == 0) v.stats[c * 8 + 7] = (int)(__builtin_amdgcn_s_memtime() - tw);
  if (lane == 0) out[c] = s;
}

}  // namespace

// the workspace layout (seqsum_bytes sizes it for 4 chains)
static size_t sq_layout(SqView& v, int64_t n, int nch, char* base) {
  v.n = n;
  v.nb = (int)((n + kSqB - 1) / kSqB);
  v.nsb = (v.nb + kSqS - 1) / kSqS;
  v.nch = nch;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* q = base + off;
    off += (bytes + 255) & ~(size_t)255;
    return q;
  };
  v.tot = (double*)take(sizeof(double) * nch * v.nb);
  v.pre = (double*)take(sizeof(double) * nch * v.nb);
  v.flg = (int*)take(sizeof(int) * nch * v.nb);
  v.brec = (int4*)take(sizeof(int4) * 2 * 3 * nch * (size_t)v.nb);
  v.srec = (int4*)take(sizeof(int4) * 2 * 3 * nch * (size_t)v.nsb);
  v.sflg = (int*)take(sizeof(int) * nch * v.nsb);
  v.soa = (float*)take(sizeof(float) * nch * (size_t)v.nb * kSqB);
  return off;
}

size_t seqsum_bytes(int64_t n) {
  SqView v;
  return sq_layout(v, std::max<int64_t>(n, 1), 4, nullptr);
}

// out[c] for c < nch: the sequential float sum of component c of x[0..n)
int seqsum_enqueue(const float4* d_x, int64_t n, int nch, void* ws, float* d_out, hipStream_t st,
                   int* d_stats) {
  if (nch < 1 || nch > 4 || n < 0) return RST_E_ARG;
  if (n == 0) {
    RST_HIP(hipMemsetAsync(d_out, 0, sizeof(float) * nch, st));
    return RST_OK;
  }
  if (n > (int64_t)INT_MAX) return RST_E_ARG;
  SqView v;
  sq_layout(v, n, nch, (char*)ws);
  v.stats = d_stats;
  if (d_stats) RST_HIP(hipMemsetAsync(d_stats, 0, sizeof(int) * 8 * nch, st));
  const int g4 = (v.nb + 3) / 4, gs = (v.nsb + 3) / 4;
  k_sq_tot<<<g4, 256, 0, st>>>(d_x, v);
  k_sq_scan<<<1, kScanT, 0, st>>>(v);
  k_sq_blocks<<<g4, 256, 0, st>>>(d_x, v);
  k_sq_super<<<gs, 256, 0, st>>>(v);
  k_sq_walk<<<nch, kWave, 0, st>>>(d_x, v, d_out);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

}  // namespace rst
