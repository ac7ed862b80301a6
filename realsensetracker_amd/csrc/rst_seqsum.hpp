// rst_seqsum.hpp -- the arithmetic of the parallel bit-exact sequential float
// sums (seqsum.hip), host- and device-callable so that a host emulation of
// the kernels (tests/cpp/seqsum_emu.cpp) runs the very same code on the CPU.
//
// The chain: s_0 = +0, s_{k+1} = fl(s_k + x_k) in float32, round to nearest
// even -- `dst_mean += dst.GetPoint(j)` / `cost += dist_sqr`
// (align_icp.cpp:113,120) and ComputeCentroid's loop
// (point_cloud_utils.cpp:94-96).
//
// Offset rule.  Run a stretch of the chain from a candidate start c and
// record every exact intermediate y_k = s_k + x_k and its rounding
// r_k = fl(y_k).  Start instead from c + d: if at every step
//   * a rounding step (y_k not representable): y_k + d lies in y_k's binade
//     and d is a multiple of that binade's grid g (2g when y_k is a tie),
//   * an exact step (y_k representable): y_k + d is representable too,
// then every step rounds alike, s_k(c + d) = s_k(c) + d, and the stretch
// ends at E + d.  The set of such d, intersected over the stretch, is an
// interval [LO, HI] on a lattice L = 2^need (need = the largest grid the
// stretch rounds on).  A stretch whose start is only known approximately is
// therefore run from the 2^m candidates G + r 2^e0 (r < 2^m, 2^(e0+m) >= L):
// the true start S picks r = ((S - G) / 2^e0) mod 2^m and d = S - G - r 2^e0,
// a multiple of L; if d is inside [LO_r, HI_r] the end is E_r + d, exactly.
// Maps of consecutive stretches compose the same way (a node's lanes carry
// exact values from their candidates through the children's maps, the
// window intersecting as it goes), so the chain becomes a walk over a few
// dozen verified jumps.  A failed check only costs a descent to smaller
// stretches or, at the bottom, the reference's own adds -- a result never
// depends on a guess.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RST_SQ_HD __host__ __device__ __forceinline__
#else
#define RST_SQ_HD inline
#endif

namespace rst {
namespace sq {

constexpr int kW = 16;                  // elements per block window
constexpr int kGW = 16;                 // blocks per group window
constexpr int kKW = 16;                 // groups per superblock window
constexpr int kTile = kW * kGW * kKW;   // 4096 elements: one superblock window
constexpr int kBlocksPerTile = kGW * kKW;
constexpr int kMaxSbBlocks = 2 * kBlocksPerTile - 1;  // a superblock spans <= 511 blocks
constexpr int kMaxSbElems = kMaxSbBlocks * kW + kW;   // ... and < 8208 elements
constexpr int kMaxSbGroups = 2 * kKW - 1;             // ... and <= 31 groups

// the positions of a 16-wide window a block / group / superblock may start
// at (the largest |prefix| among them): the middle of the window, so sizes
// stay within ~1.5x of the mean (r03: the map kernel follows its largest
// superblock and group; 0..15, any position, measured slower)
#ifndef RST_SQ_JLO
#define RST_SQ_JLO 4
#endif
#ifndef RST_SQ_JHI
#define RST_SQ_JHI 11
#endif
constexpr int kJLo = RST_SQ_JLO, kJHi = RST_SQ_JHI;

constexpr int kLeafM = 2, kLeafR = 1 << kLeafM;     // residues of a block map
constexpr int kGroupM = 4, kGroupR = 1 << kGroupM;  // of a group map
constexpr int kSbM = 6, kSbR = 1 << kSbM;           // of a superblock map

constexpr int kOpaque = 1;     // map flag: no map (non-finite / out-of-range values)
constexpr int kNoNeed = -100000;

// map header + per-residue entries
struct MapHdr {
  float G;    // candidate base: candidates G + r 2^e0, r < 2^m
  int e0;
  int m;
  int flags;
};
struct MapEnt {
  float E;
  int LOu, HIu;  // window, grid units; empty (LOu > HIu) = no map for this residue
};
struct Leaf {  // 16 dwords
  MapHdr h;
  MapEnt e[kLeafR];
};
struct GroupMap {  // 4 + 48 = 52 dwords, padded to 64
  MapHdr h;
  MapEnt e[kGroupR];
  int pad[12];
};
struct SbMap {  // 4 + 192 + 6 = 202 dwords, padded to 256
  MapHdr h;
  MapEnt e[kSbR];
  // the superblock's group, block and element ranges [ga, gb), [ba, bb),
  // [ea, eb): the walk's descent loads everything below it in one trip
  int ga, gb, ba, bb, ea, eb;
  int pad[54];
};

RST_SQ_HD uint32_t f2u(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __float_as_uint(f);
#else
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
#endif
}
RST_SQ_HD float u2f(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __uint_as_float(u);
#else
  float f;
  std::memcpy(&f, &u, 4);
  return f;
#endif
}
RST_SQ_HD int imax(int a, int b) { return a > b ? a : b; }
RST_SQ_HD int imin(int a, int b) { return a < b ? a : b; }
// 2^e as a float, e in [-126, 127]
RST_SQ_HD float pow2f(int e) { return u2f((uint32_t)(e + 127) << 23); }
RST_SQ_HD int ctz32(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_ctz(v);
#else
  return __builtin_ctz(v);
#endif
}

// the grid exponent of a candidate base: g0 = 2^e0 = the ulp of G's binade
// (2^-149 for zero / subnormal G)
RST_SQ_HD int grid_exp(float G) {
  const int E = (int)((f2u(G) >> 23) & 0xffu);
  return E == 0 ? -149 : E - 127 - 23;
}

// A candidate base from a guess: +0 for zero, and a positive guess so close
// to the top of its binade that G + (R - 1) g0 would leave it moves down
// (every candidate must be a float on the grid 2^e0).
RST_SQ_HD float candidate_base(float G, int R) {
  if (G == 0.0f || !(G == G) || std::isinf(G)) return 0.0f;
  const uint32_t u = f2u(G);
  const int E = (int)((u >> 23) & 0xffu);
  if (E == 0 || E >= 254 || (u >> 31)) return G;  // subnormal / huge / negative: stays
  const uint32_t top = (uint32_t)(E + 1) << 23;   // 2^(e+1)
  return (f2u(G) + (uint32_t)(R - 1) >= top) ? u2f(top - (uint32_t)R) : G;
}

// One step of a monitored run: s <- fl(s + x), intersecting the offset
// window [lo, hi] and raising `need` (the lattice exponent) per the offset
// rule above.  e0: the run's candidate grid exponent.  Every bound is
// computed exactly in float (each is a multiple of the step's grid within
// 24 bits of it) and errs toward a narrower window.
struct Run {
  float s, lo, hi;
  int need;
  bool opaque;
};

RST_SQ_HD void run_init(Run& p, float s0) {
  p.s = s0;
  p.lo = -INFINITY;
  p.hi = INFINITY;
  p.need = kNoNeed;
  p.opaque = false;
}

// (branch-free: every case's bounds computed, then selected -- the leaf
// runs of a wavefront take different cases in the same step; the values
// are those of the case analysis in the comments)
RST_SQ_HD void run_step(Run& p, float x, int e0) {
  const float s = p.s;
  const float r = s + x;
  // Fast2Sum on ordered operands: y = r + err exactly
  const bool sbig = fabsf(s) >= fabsf(x);
  const float a = sbig ? s : x, b = sbig ? x : s;
  const float z = r - a;
  const float err = b - z;
  p.s = r;
  const uint32_t bits = f2u(r);
  const int Er = (int)((bits >> 23) & 0xffu);
  const uint32_t man = bits & 0x7fffffu;
  const bool neg = (bits >> 31) != 0;
  // +-0 result: exact cancellation (anything else would be subnormal); the
  // window +-2^(e0+24), no lattice need, opaque unless exact
  const bool zero = r == 0.0f;
  // else |r| in [2^-99, 2^126): normal grids far from under/overflow, else no map
  const bool bad = !zero && (Er < 28 || Er > 252 || !(err == err));
  const bool inexact = err != 0.0f;
  const int er = Er - 127;
  // y's binade: below |r| when r is a power of two rounded up from beneath
  const bool below = man == 0 && inexact && ((f2u(err) >> 31) != (bits >> 31));
  const int ey = below ? er - 1 : er;
  // inexact: magnitude offsets dm with |y| + dm in [2^ey, 2^(ey+1)), dm a
  // multiple of gy
  const float gy = pow2f(ey - 23);
  const float ra = fabsf(r);
  const float ea = neg ? -err : err;   // |y| = ra + ea
  const float D = pow2f(ey) - ra;      // <= 0
  const float U = pow2f(ey + 1) - ra;  // >= 0
  const float lo_m = ea > 0.0f ? D : D + gy;
  const float hi_m = ea < 0.0f ? U : U - gy;
  const bool tie = fabsf(err) == 0.5f * gy;
  // exact: y + d stays representable while |y + d| <= 2^24 q,
  // q = min(lsb(y), max(g0, grid(y))) (the lattice is raised to grid(y))
  const int elsb = er - 23 + ctz32(man | 0x800000u);
  const int eq = imin(elsb, imax(e0, ey - 23));
  const float B = pow2f(imin(eq + 24, 127));
  const float B0 = pow2f(imin(e0 + 24, 127));
  float wlo = inexact ? (neg ? -hi_m : lo_m) : (neg ? -B - r : -B);
  float whi = inexact ? (neg ? -lo_m : hi_m) : (neg ? B : B - r);
  wlo = zero ? -B0 : wlo;
  whi = zero ? B0 : whi;
  const int nd = ey - 23 + (inexact && tie ? 1 : 0);
  p.opaque = p.opaque || bad || (zero && inexact);
  p.lo = bad ? p.lo : fmaxf(p.lo, wlo);
  p.hi = bad ? p.hi : fminf(p.hi, whi);
  p.need = bad || zero ? p.need : imax(p.need, nd);
}

// Windows are stored in units of the map's grid 2^e0, clamped to
// +-2^24 units (rounded inward: a clamp only narrows a window).
constexpr int kWinMax = 1 << 24;
RST_SQ_HD int lo_units(double lo, int e0) {
  const double u = std::ceil(std::ldexp(lo, -e0));
  if (!(u > -(double)kWinMax)) return -kWinMax;
  if (u > (double)kWinMax) return kWinMax + 1;  // empty
  return (int)u;
}
RST_SQ_HD int hi_units(double hi, int e0) {
  const double u = std::floor(std::ldexp(hi, -e0));
  if (!(u < (double)kWinMax)) return kWinMax;
  if (u < -(double)kWinMax) return -kWinMax - 1;  // empty
  return (int)u;
}

// k = (v - G) / 2^e0 for an exact value v: from the bits when v has G's
// sign and binade (G normal, e0 its grid: the usual case), else in exact
// double arithmetic.  False when v is not on the grid, non-finite, or
// implausibly far from G.
// (the exact double path: v in another binade than G; by value in and out:
// a reference argument to an out-of-line call would put the caller's
// header and k on the stack)
struct OffK {
  int ok, k;
};
#if defined(__HIPCC__) && !defined(RST_SQ_SLOW_INLINE)
__host__ __device__ __noinline__
#elif defined(__HIPCC__)
__host__ __device__ __forceinline__
#else
inline
#endif
OffK offset_units_slow(float v, float G, int e0) {
  if (!(v - v == 0.0f)) return OffK{0, 0};
  const double kv = std::ldexp((double)v, -e0);
  const double kg = std::ldexp((double)G, -e0);
  if (kv != std::floor(kv)) return OffK{0, 0};
  const double kd = kv - kg;
  if (!(std::fabs(kd) < 1073741824.0)) return OffK{0, 0};
  return OffK{1, (int)kd};
}
RST_SQ_HD bool offset_units(float v, const MapHdr& h, int& k) {
  const uint32_t vb = f2u(v), gb = f2u(h.G);
  if (((vb ^ gb) >> 23) == 0) {
    const int d = (int)(vb & 0x7fffffu) - (int)(gb & 0x7fffffu);
    k = (gb >> 31) ? -d : d;
    return true;
  }
  const OffK o = offset_units_slow(v, h.G, h.e0);
  k = o.k;
  return o.ok != 0;
}
// the bits path only (false in another binade: the caller takes its slow path)
RST_SQ_HD bool offset_units_fast(float v, const MapHdr& h, int& k) {
  const uint32_t vb = f2u(v), gb = f2u(h.G);
  if (((vb ^ gb) >> 23) == 0) {
    const int d = (int)(vb & 0x7fffffu) - (int)(gb & 0x7fffffu);
    k = (gb >> 31) ? -d : d;
    return true;
  }
  return false;
}

// The end of a map run from the exact start G + k 2^e0: entry r = k mod
// 2^m, lattice offset du = k - r grid units; valid while du is inside the
// entry's window, then E + du 2^e0 exactly (a float add: the sum is a
// float when the map is right -- the Fast2Sum check keeps a wrong map
// from ever producing a value).
RST_SQ_HD bool apply_ent(int du, int e0, const MapEnt& en, float& out) {
  if (!(en.LOu <= du && du <= en.HIu)) return false;
  if (du == 0) {
    out = en.E;
    return true;
  }
  const float d = std::ldexp((float)du, e0);
  const float o = en.E + d;
  const bool ebig = std::fabs(en.E) >= std::fabs(d);
  if (ebig ? (o - en.E != d) : (o - d != en.E)) return false;
  out = o;
  return true;
}

// One composite lane: the exact value v (one candidate start of a node)
// through a child map (header h, entries e[] by residue); the node's window
// [clo, chi] (absolute offsets of the node's start) narrows.  False: this
// candidate cannot pass the child.
// (in two parts for callers that fetch the entry themselves: the offset
// k of v in the child's grid, then the child's entry r = k mod 2^m applied)
RST_SQ_HD bool through_off(float v, const MapHdr& h, int mmax, int& k) {
  if ((h.flags & kOpaque) || h.m < 0 || h.m > mmax) return false;
  return offset_units(v, h, k);
}
RST_SQ_HD bool through_ent(float& v, double& clo, double& chi, const MapHdr& h, int k, const MapEnt& en) {
  const int du = k - (k & ((1 << h.m) - 1));
  float out;
  if (!apply_ent(du, h.e0, en, out)) return false;
  clo = std::fmax(clo, std::ldexp((double)(en.LOu - du), h.e0));
  chi = std::fmin(chi, std::ldexp((double)(en.HIu - du), h.e0));
  v = out;
  return true;
}
RST_SQ_HD bool through(float& v, double& clo, double& chi, const MapHdr& h, const MapEnt* e) {
  int k;
  if (!through_off(v, h, kSbM, k)) return false;
  return through_ent(v, clo, chi, h, k, e[k & ((1 << h.m) - 1)]);
}

}  // namespace sq
}  // namespace rst
