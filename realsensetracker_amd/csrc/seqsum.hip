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
// {lo1, hi0, hi1, problem}
struct Fn {
  int d[2], lo[2], hi[2];
};

__device__ __forceinline__ Fn fn_ident() {
  Fn f;
  f.d[0] = f.d[1] = 0;
  f.lo[0] = f.lo[1] = kInv;
  f.hi[0] = f.hi[1] = -kInv;
  return f;
}
__device__ __forceinline__ Fn fn_invalid() {
  Fn f;
  f.d[0] = f.d[1] = 0;
  f.lo[0] = f.lo[1] = -kInv;
  f.hi[0] = f.hi[1] = kInv;
  return f;
}

// f then g
__device__ __forceinline__ Fn fn_compose(const Fn& f, const Fn& g) {
  Fn h;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int fd = f.d[p];
    const int q = (p + fd) & 1;
    int d = fd + g.d[q];
    int lo = min(f.lo[p], fd + g.lo[q]);
    int hi = max(f.hi[p], fd + g.hi[q]);
    if (lo < -kLim || hi > kLim || d > kLim || d < -kLim) {  // saturate: never valid
      d = 0;
      lo = -kInv;
      hi = kInv;
    }
    h.d[p] = d;
    h.lo[p] = lo;
    h.hi[p] = hi;
  }
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
  Fn f;
  const int hi = a + (fr > 0.0 ? 1 : 0);
  f.lo[0] = f.lo[1] = a;
  f.hi[0] = f.hi[1] = hi;
  if (fr == 0.5) {  // tie: the even result
    f.d[0] = a + ((0 + a) & 1);
    f.d[1] = a + ((1 + a) & 1);
  } else {
    f.d[0] = f.d[1] = a + (fr > 0.5 ? 1 : 0);
  }
  return f;
}

__device__ __forceinline__ Fn fn_shfl_down(const Fn& f, int o) {
  Fn g;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    g.d[p] = __shfl_down(f.d[p], o, kWave);
    g.lo[p] = __shfl_down(f.lo[p], o, kWave);
    g.hi[p] = __shfl_down(f.hi[p], o, kWave);
  }
  return g;
}
__device__ __forceinline__ Fn fn_shfl_up(const Fn& f, int o) {
  Fn g;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    g.d[p] = __shfl_up(f.d[p], o, kWave);
    g.lo[p] = __shfl_up(f.lo[p], o, kWave);
    g.hi[p] = __shfl_up(f.hi[p], o, kWave);
  }
  return g;
}

// ordered composition of the wave's 64 maps (lane 0 first); lane 0 gets it
__device__ __forceinline__ Fn fn_wave_reduce(Fn f, int lane) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const Fn g = fn_shfl_down(f, o);
    if ((lane & (2 * o - 1)) == 0) f = fn_compose(f, g);
  }
  return f;
}
// inclusive ordered prefix: lane j gets map_0 then ... then map_j
__device__ __forceinline__ Fn fn_wave_scan(Fn f, int lane) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const Fn g = fn_shfl_up(f, o);
    if (lane >= o) f = fn_compose(g, f);
  }
  return f;
}

__device__ __forceinline__ int slot_of(int e) { return ((e % 3) + 3) % 3; }

__device__ __forceinline__ void rec_store(int4* rec, int e, const Fn& f, int problem) {
  rec[0] = make_int4(e, f.d[0], f.d[1], f.lo[0]);
  rec[1] = make_int4(f.lo[1], f.hi[0], f.hi[1], problem);
}
__device__ __forceinline__ Fn rec_fn(int4 a, int4 b) {
  Fn f;
  f.d[0] = a.y;
  f.d[1] = a.z;
  f.lo[0] = a.w;
  f.lo[1] = b.x;
  f.hi[0] = b.y;
  f.hi[1] = b.z;
  return f;
}

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

// non-finite flags of a value: 1 NaN, 2 +inf, 4 -inf
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
    const int fl = nf_flags(xc);
    const double s = wave_sum(fl ? 0.0 : (double)xc);
    const int f = (__ballot(fl & 1) ? 1 : 0) | (__ballot(fl & 2) ? 2 : 0) | (__ballot(fl & 4) ? 4 : 0);
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
      f = fn_wave_reduce(f, lane);
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
      f = fn_wave_reduce(f, lane);
      if (lane == 0) rec_store(srec + ((int64_t)s * v.nsb + sb) * 2, e, f, 0);
    }
    if (lane == 0) v.sflg[(int64_t)c * v.nsb + sb] = orf;
  }
}

// ---- 5: the walk (one wavefront per chain) ----------------------------------------------
// Try to jump over up to `cnt` consecutive units (superblocks or blocks) whose
// records for binade e start at rec (stride 2 int4 per unit), from the true
// s.  Returns the number of units jumped (0: none) and updates s.
__device__ __forceinline__ int try_jump(const int4* __restrict__ rec, int cnt, int e, bool stop_problem,
                                        float& s, int lane) {
  Fn f;
  bool ok = false;
  if (lane < cnt) {
    const int4 r0 = rec[2 * lane], r1 = rec[2 * lane + 1];
    ok = r0.x == e && !(stop_problem && r1.w && lane > 0);
    f = ok ? rec_fn(r0, r1) : fn_invalid();
  } else {
    f = fn_invalid();
  }
  // lanes after the first unusable unit cannot be reached
  const uint64_t bad = __ballot(!ok);
  const int first_bad = bad ? __builtin_ctzll(bad) : kWave;
  if (first_bad == 0) return 0;
  f = fn_wave_scan(f, lane);
  const uint32_t bits = __float_as_uint(s);
  const int S0 = (int)((bits & 0x7fffffu) | 0x800000u);
  const int S = (bits >> 31) ? -S0 : S0;
  const int p = S & 1;
  const int dd = f.d[p], lo = f.lo[p], hi = f.hi[p];
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

__global__ __launch_bounds__(kWave) void k_sq_walk(const float4* __restrict__ x, SqView v,
                                                   float* __restrict__ out) {
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  const int4* brec = v.brec + ((int64_t)c * 3) * v.nb * 2;
  const int4* srec = v.srec + ((int64_t)c * 3) * v.nsb * 2;
  float s = 0.0f;
  int b = 0;
  while (b < v.nb) {
    if (!isfinite(s)) {
      // inf / NaN absorbs every finite element: only NaN or an opposite
      // infinity in the rest can still change it
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
      if ((b % kSqS) == 0) {  // superblocks
        const int sb = b / kSqS;
        const int cnt = min(kWave, v.nsb - sb);
        const int k = try_jump(srec + ((int64_t)sl * v.nsb + sb) * 2, cnt, e, false, s, lane);
        if (k > 0) {
          b = min(v.nb, b + k * kSqS);
          continue;
        }
      }
      // blocks, up to the next superblock boundary
      const int cnt = min(kSqS - (b % kSqS), v.nb - b);
      const int4* r = brec + ((int64_t)sl * v.nb + b) * 2;
      const bool first_problem = r[1].w != 0;
      if (!first_problem) {
        const int k = try_jump(r, cnt, e, true, s, lane);
        if (k > 0) {
          b += k;
          continue;
        }
      }
    }
    // one block in the reference's order
    const int64_t i0 = (int64_t)b * kSqB;
    const int m = (int)min<int64_t>(kSqB, v.n - i0);
    const float xv = lane < m ? comp(x[i0 + lane], c) : 0.0f;
    for (int k = 0; k < m; ++k) s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), k));
    ++b;
  }
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
  return off;
}

size_t seqsum_bytes(int64_t n) {
  SqView v;
  return sq_layout(v, std::max<int64_t>(n, 1), 4, nullptr);
}

// out[c] for c < nch: the sequential float sum of component c of x[0..n)
int seqsum_enqueue(const float4* d_x, int64_t n, int nch, void* ws, float* d_out, hipStream_t st) {
  if (nch < 1 || nch > 4 || n < 0) return RST_E_ARG;
  if (n == 0) {
    RST_HIP(hipMemsetAsync(d_out, 0, sizeof(float) * nch, st));
    return RST_OK;
  }
  if (n > (int64_t)INT_MAX) return RST_E_ARG;
  SqView v;
  sq_layout(v, n, nch, (char*)ws);
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
