// rst_wave_nn.hpp -- exact 1-NN for a wavefront of spatially coherent
// queries (the ICP hot loop, align_icp.cpp:105-121 / kdtree.hpp:51-57).
//
// Why a wave-level search: per-lane tree walks gather a different BVH node
// per lane at every step (64 cache lines per wave instruction), which
// saturates the texture path long before HBM; a wave-uniform walk with
// scalar loads serialises ~hundreds of dependent loads.  Here the 64 queries
// of a wave (Morton-consecutive source points, one compact surface patch)
// share ONE staging walk and then search the staged leaves from registers:
//
//   1. every lane has a bound: the d2 of its warm candidate (last
//      iteration's neighbour; cold lanes take the best point of the leaf a
//      greedy near-child descent reaches);
//   2. regions = AABB of the balls (radius sqrt(bound), inflated) of each
//      8-lane group, and their union;
//   3. staging walk: LIFO stack of node ids in LDS, popped up to 64 at a
//      time -- lane t loads node t's box (one coalesced load per round, all
//      in flight together), keeps it if it meets a group region; internal nodes
//      push both children, leaves are staged (box + id) in LDS.  The walk
//      starts at the lowest common ancestor of the lanes' start leaves plus
//      the sibling of every ancestor, i.e. still the whole tree;
//   4. flush (every <= 64 staged leaves, and at the end): leaves any lane's
//      ball touches (per-lane box test, ballot) are loaded four at a time,
//      one 16-point leaf per 16 lanes in a single load instruction, and
//      each point is broadcast to all lanes with v_readlane; every lane
//      offers it to its own lexicographic (d2, index) minimum.  The region
//      shrinks after every flush as the bounds tighten.
//
// Exactness: a node is dropped only if its box misses every group region,
// i.e. for every lane its box_d2 exceeds that lane's bound; a staged leaf is skipped
// only if no lane's box_d2 <= bound.  Bounds only decrease, so every point
// not offered is strictly worse than the final answer (same argument as the
// tree walks of rst_bvh.hpp, which tests/cpp/bvh_selftest.cpp checks).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>

#include "rst_bvh.hpp"
#include "rst_device.hpp"

namespace rst {

constexpr int kWnnStack = 512;   // node ids per wave (see the overflow rule)
constexpr int kWnnLeaves = 128;  // staged leaves per flush
constexpr int kWnnPop = 64;      // nodes tested per staging round
constexpr int kWnnGroups = 8;    // lane groups with their own region (8 lanes each)
// Work cap of the shared walk: a wave whose regions stage more leaves than
// this (a cold start with poor seeds, a cluster of far outliers) finishes
// with per-lane bottom-up searches instead (rst_bvh.hpp search_from: exact
// from any starting bound; divergent gathers, but a bounded latency chain).
constexpr int kWnnCap = 256;

// Lanes of one wavefront hand data to each other through LDS (WnnScratch)
// between these points.  The hardware executes a wave's LDS accesses in
// order, but the compiler may move plain memory operations across a bare
// wave_barrier (and across wavefront-scope fences, which order atomics
// only); the asm memory clobber pins them.  No cache maintenance.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // a full compiler barrier for plain (non-atomic) LDS accesses too, and
  // every LDS access of this wave retired before the next one issues
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

struct WnnScratch {              // per-wave LDS (6.6 KB)
  int stack[kWnnStack];
  float4 leaf_lo[kWnnLeaves];    // .w = leaf index bits
  float4 leaf_hi[kWnnLeaves];
  float4 greg_lo[2 * kWnnGroups];  // AABBs of the group's ordinary balls (2 runs)
  float4 greg_hi[2 * kWnnGroups];
  float4 gsph[kWnnGroups];       // sphere around the group's big balls (xyz, R^2)
};

// A lane whose bound exceeds this radius (metres) is "big": its ball joins
// its group's bounding sphere instead of the group's AABB.  An off-surface
// query (frame border, occlusion) has a large ball that touches the target
// surface only near its neighbour; the ball's AABB would take in a whole
// square of surface, a sphere test does not.
constexpr float kWnnBigR = 0.012f;
// A group whose largest step between consecutive queries exceeds this
// (metres) straddles a jump of the Morton curve (e.g. far wall -> near
// object): its ordinary balls get one AABB per side of the jump.
constexpr float kWnnJump = 0.05f;

// Butterfly partners without LDS: the value of lane l's partner at level K
// of an ASCENDING reduction -- K = 0, 1: l ^ 1, l ^ 2 (DPP quad_perm);
// K = 2, 3: 7 - l within the half row, 15 - l within the row (DPP
// row_half_mirror / row_mirror); K = 4, 5: the other row of the pair, the
// other half of the wave (v_permlane16_swap / v_permlane32_swap).  After
// levels 0..K-1 every aligned group of 2^K lanes holds one value, so the
// mirror partner stands for the xor one; valid for merges that are
// commutative, associative and idempotent (min, max, lexicographic top-k),
// whose result does not depend on the order.  The whole wave must be active.
// (r19: a ds_bpermute per exchange put an LDS round trip on every step of
// the searches' wave reductions)
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
template <int K>
__device__ __forceinline__ int bfly(int x) {
  static_assert(K >= 0 && K <= 5, "levels 0..5 of a wave of 64");
  if constexpr (K == 0) {
    return dpp_i<kDppXor1>(x);
  } else if constexpr (K == 1) {
    return dpp_i<kDppXor2>(x);
  } else if constexpr (K == 2) {
    return dpp_i<kDppRowHalfMirror>(x);
  } else if constexpr (K == 3) {
    return dpp_i<kDppRowMirror>(x);
  } else if constexpr (K == 4) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    return (__lane_id() & 16) ? (int)r[0] : (int)r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    return (__lane_id() & 32) ? (int)r[0] : (int)r[1];
  }
}
template <int K>
__device__ __forceinline__ float bfly(float x) {
  return i2f(bfly<K>(f2i(x)));
}
// v <- op(v, partner) for levels 0 .. L-1 (L = 6: the wave, 4: rows of 16,
// 3: groups of 8)
template <int L, class T, class Op>
__device__ __forceinline__ T bfly_reduce(T v, Op op) {
  if constexpr (L > 0) v = op(v, bfly<0>(v));
  if constexpr (L > 1) v = op(v, bfly<1>(v));
  if constexpr (L > 2) v = op(v, bfly<2>(v));
  if constexpr (L > 3) v = op(v, bfly<3>(v));
  if constexpr (L > 4) v = op(v, bfly<4>(v));
  if constexpr (L > 5) v = op(v, bfly<5>(v));
  return v;
}
struct OpMinI {
  __device__ int operator()(int a, int b) const { return min(a, b); }
};
struct OpMaxI {
  __device__ int operator()(int a, int b) const { return max(a, b); }
};
struct OpMinF {
  __device__ float operator()(float a, float b) const { return fminf(a, b); }
};
struct OpMaxF {
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};

__device__ __forceinline__ float wnn_rl(float v, int l) {
  return i2f(__builtin_amdgcn_readlane(f2i(v), l));
}
__device__ __forceinline__ int wnn_min_i(int v) { return bfly_reduce<6>(v, OpMinI{}); }
__device__ __forceinline__ int wnn_max_i(int v) { return bfly_reduce<6>(v, OpMaxI{}); }
__device__ __forceinline__ float wnn_min_f(float v) { return bfly_reduce<6>(v, OpMinF{}); }
__device__ __forceinline__ float wnn_max_f(float v) { return bfly_reduce<6>(v, OpMaxF{}); }

// Cold lane: follow near children to one leaf and take its best point as
// the starting bound (any real point will do; exactness comes later).
__device__ __forceinline__ void wnn_seed(const BvhView& bv, float qx, float qy, float qz,
                                         Best1& r) {
  int k = 1;
  while (k < bv.nleaves) {
    const float4 lo = bv.nodes[2 * k];
    const float4 hi = bv.nodes[2 * k + 1];
    k = near_child(k, lo, hi, qx, qy, qz);
  }
  scan_leaf(bv, k - bv.nleaves, qx, qy, qz, r);
}

struct WnnRegion {
  float lx, ly, lz, hx, hy, hz;
  __device__ __forceinline__ bool meets(const float4& lo, const float4& hi) const {
    return lo.x <= hx && hi.x >= lx && lo.y <= hy && hi.y >= ly && lo.z <= hz && hi.z >= lz;
  }
};

// min / max over the 8 lanes of a group (levels 0-2 stay in the group)
__device__ __forceinline__ float wnn_gmin(float v) { return bfly_reduce<3>(v, OpMinF{}); }
__device__ __forceinline__ float wnn_gmax(float v) { return bfly_reduce<3>(v, OpMaxF{}); }

// Regions of the current bounds, per 8-lane group (in LDS): the AABB of the
// ordinary balls -- two AABBs, one per side, when the group straddles a
// jump of the Morton curve -- and a sphere holding the big balls (a far
// outlier only widens its own group's sphere); the union AABB is returned.
__device__ __forceinline__ WnnRegion wnn_regions(bool act, float qx, float qy, float qz,
                                                 float bound, WnnScratch& ws) {
  // inflate so float rounding can never drop a node some lane needs
  const float rad = act ? sqrtf(bound) * 1.0001f + 1e-20f : 0.0f;
  const bool big = act && rad > kWnnBigR;
  const bool ord = act && !big;
  const int lane = __lane_id();
  const int gl = lane & 7;
  // largest step to the previous query inside the group -> run split point
  const float px = __shfl(qx, lane - 1, 64), py = __shfl(qy, lane - 1, 64),
              pz = __shfl(qz, lane - 1, 64);
  const bool pact = __shfl((int)act, lane - 1, 64) != 0;
  float gap = -1.f;
  if (gl > 0 && act && pact) {
    const float ex = qx - px, ey = qy - py, ez = qz - pz;
    gap = ex * ex + ey * ey + ez * ez;
  }
  float gbest = gap;
  int gk = gl;
  // (the group's largest gap, lowest index on ties: a total order, so the
  // butterfly's pairing does not matter)
  auto gstep = [&](float og, int ok) {
    const bool take = (og > gbest) | ((og == gbest) & (ok < gk));
    gbest = take ? og : gbest;
    gk = take ? ok : gk;
  };
  gstep(bfly<0>(gbest), bfly<0>(gk));
  gstep(bfly<1>(gbest), bfly<1>(gk));
  gstep(bfly<2>(gbest), bfly<2>(gk));
  const int run = (gbest > kWnnJump * kWnnJump && gl >= gk) ? 1 : 0;
  float lx[2], ly[2], lz[2], hx[2], hy[2], hz[2];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    const bool in = ord && run == sub;
    lx[sub] = wnn_gmin(in ? qx - rad : FLT_MAX);
    ly[sub] = wnn_gmin(in ? qy - rad : FLT_MAX);
    lz[sub] = wnn_gmin(in ? qz - rad : FLT_MAX);
    hx[sub] = wnn_gmax(in ? qx + rad : -FLT_MAX);
    hy[sub] = wnn_gmax(in ? qy + rad : -FLT_MAX);
    hz[sub] = wnn_gmax(in ? qz + rad : -FLT_MAX);
  }
  // big balls: centre = middle of their centres, R = max |q - c| + r
  const float bx0 = wnn_gmin(big ? qx : FLT_MAX), bx1 = wnn_gmax(big ? qx : -FLT_MAX);
  const float by0 = wnn_gmin(big ? qy : FLT_MAX), by1 = wnn_gmax(big ? qy : -FLT_MAX);
  const float bz0 = wnn_gmin(big ? qz : FLT_MAX), bz1 = wnn_gmax(big ? qz : -FLT_MAX);
  const bool anybig = bx0 <= bx1;
  const float cx = anybig ? 0.5f * (bx0 + bx1) : 0.f;
  const float cy = anybig ? 0.5f * (by0 + by1) : 0.f;
  const float cz = anybig ? 0.5f * (bz0 + bz1) : 0.f;
  const float dx = qx - cx, dy = qy - cy, dz = qz - cz;
  const float R = wnn_gmax(big ? (sqrtf(dx * dx + dy * dy + dz * dz) + rad) * 1.0001f + 1e-20f
                               : 0.f);
  if (gl == 0) {
    const int g = lane >> 3;
    ws.greg_lo[2 * g] = make_float4(lx[0], ly[0], lz[0], 0.f);
    ws.greg_hi[2 * g] = make_float4(hx[0], hy[0], hz[0], 0.f);
    ws.greg_lo[2 * g + 1] = make_float4(lx[1], ly[1], lz[1], 0.f);
    ws.greg_hi[2 * g + 1] = make_float4(hx[1], hy[1], hz[1], 0.f);
    ws.gsph[g] = make_float4(cx, cy, cz, anybig ? R * R * 1.0001f : -1.f);
  }
  WnnRegion u;
  u.lx = wnn_min_f(fminf(fminf(lx[0], lx[1]), anybig ? cx - R : FLT_MAX));
  u.ly = wnn_min_f(fminf(fminf(ly[0], ly[1]), anybig ? cy - R : FLT_MAX));
  u.lz = wnn_min_f(fminf(fminf(lz[0], lz[1]), anybig ? cz - R : FLT_MAX));
  u.hx = wnn_max_f(fmaxf(fmaxf(hx[0], hx[1]), anybig ? cx + R : -FLT_MAX));
  u.hy = wnn_max_f(fmaxf(fmaxf(hy[0], hy[1]), anybig ? cy + R : -FLT_MAX));
  u.hz = wnn_max_f(fmaxf(fmaxf(hz[0], hz[1]), anybig ? cz + R : -FLT_MAX));
  wave_sync();
  return u;
}

__device__ __forceinline__ bool wnn_meets_group(const WnnScratch& ws, const float4& lo,
                                                const float4& hi) {
  bool m = false;
#pragma unroll
  for (int k = 0; k < 2 * kWnnGroups; ++k) {
    const float4 a = ws.greg_lo[k], b = ws.greg_hi[k];
    m |= (lo.x <= b.x) & (hi.x >= a.x) & (lo.y <= b.y) & (hi.y >= a.y) & (lo.z <= b.z) &
         (hi.z >= a.z);
  }
#pragma unroll
  for (int g = 0; g < kWnnGroups; ++g) {
    const float4 c = ws.gsph[g];
    m |= box_d2(c.x, c.y, c.z, lo, hi) <= c.w;
  }
  return m;
}

// Offer the staged leaves [0, ns) to every active lane.  Four leaves per
// load instruction (lanes 16g..16g+15 hold leaf g's <= 16 points); a leaf
// whose box no lane's ball touches (bounds as of that moment) is skipped.
__device__ __forceinline__ int wnn_flush(const BvhView& bv, const WnnScratch& ws, int ns,
                                         bool act, float qx, float qy, float qz, Best1& r) {
  const int lane = __lane_id();
  int scanned = 0;
  const int g = lane >> 4, o = lane & 15;
  for (int s = 0; s < ns; s += 4) {
    int cnt = 0, b = 0;
    if (s + g < ns) {
      const int L = f2i(ws.leaf_lo[s + g].w);
      b = leaf_begin(bv, L);
      cnt = leaf_begin(bv, L + 1) - b;
    }
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (o < cnt) p = bv.pts[b + o];
    for (int gg = 0; gg < 4 && s + gg < ns; ++gg) {
      const float4 lo = ws.leaf_lo[s + gg];
      const float4 hi = ws.leaf_hi[s + gg];
      if (__ballot(act && box_d2(qx, qy, qz, lo, hi) <= r.d) == 0) continue;
      ++scanned;
      const int c = __builtin_amdgcn_readlane(cnt, 16 * gg);
      const int bb = __builtin_amdgcn_readlane(b, 16 * gg);
      for (int j = 0; j < c; ++j) {
        const int src = 16 * gg + j;
        const float px = wnn_rl(p.x, src), py = wnn_rl(p.y, src), pz = wnn_rl(p.z, src);
        const int id = __builtin_amdgcn_readlane(f2i(p.w), src);
        if (act) r.offer(d2_ref(qx, qy, qz, px, py, pz), id, bb + j);
      }
    }
  }
  return scanned;
}

// Exact 1-NN for every lane with act (the wave must be converged here).
// r arrives holding the warm candidate (or empty) and leaves with the exact
// lexicographic (d2, index) minimum; non-finite queries find nothing.
// stats (diagnostics, may be null): per wave, 8 ints at stats[8 * wave]:
// staging rounds, nodes tested, leaves staged, leaves scanned, wave time
// (s_memrealtime ticks, 10 ns), active lanes, lanes with no finite bound,
// region extent (um, max axis).
__device__ __forceinline__ void nn_wave_region(const BvhView& bv, bool act, float qx, float qy,
                                            float qz, Best1& r, WnnScratch& ws,
                                            int* stats = nullptr) {
  const int lane = __lane_id();
  const int nl = bv.nleaves;
  const uint64_t t_start = stats ? __builtin_amdgcn_s_memrealtime() : 0;
  act = act && bv.m > 0 && finite3(qx, qy, qz);
  if (act && r.pos < 0) wnn_seed(bv, qx, qy, qz, r);
  if (__ballot(act) == 0) return;
  // start: lowest common ancestor of the lanes' start leaves
  const int leaf = (act && r.pos >= 0) ? leaf_of(bv, r.pos) : -1;
  const int lmin = wnn_min_i(act && leaf >= 0 ? leaf : INT_MAX);
  const int lmax = wnn_max_i(act && leaf >= 0 ? leaf : -1);
  const bool anyempty = __ballot(act && leaf < 0) != 0;
  unsigned lca = 1;
  if (!anyempty && lmax >= 0) {
    const unsigned a = (unsigned)(nl + lmin), b = (unsigned)(nl + lmax);
    lca = (a == b) ? a : (a >> (32 - __clz(a ^ b)));
  }
  // stack = siblings of lca's ancestors (bottom) .. lca (top)
  const int depth = 31 - __clz(lca);  // levels above lca
  if (lane < depth) ws.stack[lane] = (int)((lca >> (depth - 1 - lane)) ^ 1u);
  if (lane == 0) ws.stack[depth] = (int)lca;
  int sp = depth + 1;
  wave_sync();
  WnnRegion reg = wnn_regions(act, qx, qy, qz, r.d, ws);
  int ns = 0;
  int st_rounds = 0, st_nodes = 0, st_staged = 0, st_scanned = 0, st_flush = 0;
  if (stats) {
    const int nact = __popcll(__ballot(act));
    const int ninf = __popcll(__ballot(act && !(r.d < FLT_MAX)));
    const float ext = fmaxf(fmaxf(reg.hx - reg.lx, reg.hy - reg.ly), reg.hz - reg.lz);
    if (lane == 0) {
      stats[5] = nact;
      stats[6] = ninf;
      stats[7] = (int)fminf(ext * 1e6f, 2e9f);
    }
  }
  const uint64_t lt = (1ull << lane) - 1ull;
  while (sp > 0 || ns > 0) {
    if (sp > 0) {
      // overflow rule: above the high-water mark pop one node at a time
      // (pure DFS grows the stack by at most the tree depth)
      // overflow rule: pops shrink as the stack fills, down to one node at
      // a time (pure DFS then grows the stack by at most the tree depth)
      const int k = min(min(kWnnPop, sp), max(1, (kWnnStack - 48 - sp) / 2));
      ++st_rounds;
      st_nodes += k;
      int node = 0;
      if (lane < k) node = ws.stack[sp - 1 - lane];
      sp -= k;
      wave_sync();
      bool pass = false;
      float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
      if (lane < k) {
        lo = bv.nodes[2 * node];
        hi = bv.nodes[2 * node + 1];
        pass = reg.meets(lo, hi) && wnn_meets_group(ws, lo, hi);
      }
      const bool isleaf = node >= nl;
      const uint64_t im = __ballot(pass && !isleaf);
      const uint64_t lm = __ballot(pass && isleaf);
      if (pass && !isleaf) {
        const int rk = __popcll(im & lt);
        // far child below near child: the near one is popped first
        const int nc = near_child(node, lo, hi, 0.5f * (reg.lx + reg.hx),
                                  0.5f * (reg.ly + reg.hy), 0.5f * (reg.lz + reg.hz));
        ws.stack[sp + 2 * rk] = nc ^ 1;
        ws.stack[sp + 2 * rk + 1] = nc;
      }
      if (pass && isleaf) {
        const int rk = __popcll(lm & lt);
        const int L = node - nl;
        ws.leaf_lo[ns + rk] = make_float4(lo.x, lo.y, lo.z, i2f(L));
        ws.leaf_hi[ns + rk] = hi;
      }
      sp += 2 * __popcll(im);
      ns += __popcll(lm);
      st_staged += __popcll(lm);
      wave_sync();
    }
    const bool over = st_staged > kWnnCap;
    if (ns > kWnnLeaves - kWnnPop || (ns > 0 && (sp == 0 || over))) {
      st_scanned += wnn_flush(bv, ws, ns, act, qx, qy, qz, r);
      ++st_flush;
      ns = 0;
      reg = wnn_regions(act, qx, qy, qz, r.d, ws);
    }
    if (over) {
      // fallback: every lane finishes on its own (exact from its bound)
      if (act) {
        if (r.pos >= 0)
          search_from(bv, r.pos, qx, qy, qz, r);
        else
          descend(bv, 1, qx, qy, qz, r);
      }
      st_flush = -1;
      break;
    }
  }
  if (stats && lane == 0) {
    stats[0] = st_rounds;
    stats[1] = st_nodes;
    stats[2] = st_staged;
    stats[3] = st_scanned;
    stats[4] = (int)(__builtin_amdgcn_s_memrealtime() - t_start);
    if (st_flush < 0) stats[5] = -stats[5];  // marks a capped wave
  }
}

}  // namespace rst

namespace rst {

// ---- one query, a whole wavefront ------------------------------------------------
// The fallback of the ICP search (queries the leaf adjacency cannot cover:
// cold starts with poor seeds, far outliers at frame borders and
// occlusions).  All 64 lanes work on the same query q: the staging walk
// tests up to 64 nodes per round exactly (box_d2 <= bound), starting at the
// warm leaf and the siblings of its ancestors; staged leaves are scanned 64
// points per step, one point per lane, and a lexicographic wave minimum
// after every flush tightens the shared bound.  Latency ~ the depth of the
// subtrees the ball touches, not the number of points in it.
template <int K>
__device__ __forceinline__ void lex_step1(Best1& b) {
  const float od = bfly<K>(b.d);
  const int oid = bfly<K>(b.id);
  const int op = bfly<K>(b.pos);
  const bool t = lex_less(od, oid, b.d, b.id) | ((od == b.d) & (oid == b.id) & (op > b.pos));
  b.d = t ? od : b.d;
  b.id = t ? oid : b.id;
  b.pos = t ? op : b.pos;
}
// (a total order on (d, id, pos): the minimum does not depend on the
// butterfly's pairing, bfly)
__device__ __forceinline__ Best1 wave_lex_min(Best1 b) {
  lex_step1<0>(b);
  lex_step1<1>(b);
  lex_step1<2>(b);
  lex_step1<3>(b);
  lex_step1<4>(b);
  lex_step1<5>(b);
  return b;
}

// Wave merge of Best2 lists (sorted, distinct ids within each): the merge
// is commutative, so every lane ends with the same two entries; a point
// held by both lists (same id) counts once.
// (kTop = 8: the merge within each row of 16 lanes only)
template <int K>
__device__ __forceinline__ void lex_step2(Best2& b) {
  const float od0 = bfly<K>(b.d[0]), od1 = bfly<K>(b.d[1]);
  const int oi0 = bfly<K>(b.id[0]), oi1 = bfly<K>(b.id[1]);
  const int op0 = bfly<K>(b.pos[0]), op1 = bfly<K>(b.pos[1]);
  const bool of = lex_less(od0, oi0, b.d[0], b.id[0]);  // the other list leads
  const float fd = of ? od0 : b.d[0];
  const int fi = of ? oi0 : b.id[0], fp = of ? op0 : b.pos[0];
  // second: the leader's second, or the other head (its second when the
  // two heads are the same point)
  const float wd = of ? od1 : b.d[1];
  const int wi = of ? oi1 : b.id[1], wp = of ? op1 : b.pos[1];
  const float hd = of ? b.d[0] : od0, h2d = of ? b.d[1] : od1;
  const int hi = of ? b.id[0] : oi0, h2i = of ? b.id[1] : oi1;
  const int hp = of ? b.pos[0] : op0, h2p = of ? b.pos[1] : op1;
  const bool dup = hi == fi;
  const float cd = dup ? h2d : hd;
  const int ci = dup ? h2i : hi, cp = dup ? h2p : hp;
  const bool c2 = lex_less(cd, ci, wd, wi);
  b.d[0] = fd;
  b.id[0] = fi;
  b.pos[0] = fp;
  b.d[1] = c2 ? cd : wd;
  b.id[1] = c2 ? ci : wi;
  b.pos[1] = c2 ? cp : wp;
}
// (the two smallest of the union: commutative, associative, idempotent --
// the butterfly's pairing does not matter, bfly; levels 0-3 stay in a row)
template <int kTop = 32>
__device__ __forceinline__ Best2 wave_lex_min(Best2 b) {
  static_assert(kTop == 8 || kTop == 32, "rows of 16 or the wave");
  lex_step2<0>(b);
  lex_step2<1>(b);
  lex_step2<2>(b);
  lex_step2<3>(b);
  if constexpr (kTop == 32) {
    lex_step2<4>(b);
    lex_step2<5>(b);
  }
  return b;
}

// Scan the staged leaves [0, ns) (ws.leaf_lo[s] = (box_d2, -, -, leaf bits))
// for one query: leaf ranges first (one load per leaf, all lanes), then the
// points 32 leaves at a time -- lanes 16g..16g+15 take leaf s+g's points,
// eight leaf groups' loads in flight per lane before any offer -- so a flush
// costs a couple of memory latencies, not one per four leaves.  Leaves whose
// box_d2 exceeds the current (uniform) bound are skipped.  r <- the wave
// minimum of every lane's offers.
template <class R>
__device__ __forceinline__ void wnn_scan_ranges(const BvhView& bv, WnnScratch& ws, int ns, float qx,
                                                float qy, float qz, R& mine, R& r, int variant);

template <class R>
__device__ __forceinline__ void wnn_flush_one(const BvhView& bv, WnnScratch& ws, int ns, float qx,
                                              float qy, float qz, R& mine, R& r, int variant = 0) {
  const int lane = __lane_id();
  if (variant == 2) {  // DEBUG: the original one-leaf-group-at-a-time scan
    const int g = lane >> 4, o = lane & 15;
    for (int s = 0; s < ns; s += 4) {
      if (s + g < ns) {
        const float4 e = ws.leaf_lo[s + g];
        if (e.x <= r.bound()) {
          const int L = f2i(e.w);
          const int b = leaf_begin(bv, L);
          if (o < leaf_begin(bv, L + 1) - b) {
            const float4 p = bv.pts[b + o];
            mine.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), b + o);
          }
        }
      }
    }
    r = wave_lex_min(mine);
    wave_sync();
    return;
  }
  for (int s = lane; s < ns; s += kWave) {
    const int L = f2i(ws.leaf_lo[s].w);
    const int b = leaf_begin(bv, L);
    const int e = leaf_begin(bv, L + 1);
    ws.leaf_hi[s] = make_float4(0.f, 0.f, i2f(b), i2f(e - b));
  }
  wave_sync();
  wnn_scan_ranges(bv, ws, ns, qx, qy, qz, mine, r, variant);
}

// The point scan of wnn_flush_one over staged ranges (ws.leaf_lo[s].x =
// box_d2, ws.leaf_hi[s] = (-, -, begin, count) for s < ns).
template <class R>
__device__ __forceinline__ void wnn_scan_ranges(const BvhView& bv, WnnScratch& ws, int ns, float qx,
                                                float qy, float qz, R& mine, R& r, int variant) {
  const int lane = __lane_id();
  const int g = lane >> 4, o = lane & 15;
  const float bnd = r.bound();
  const int last = bv.m - 1;
  for (int s0 = 0; s0 < ns; s0 += 32) {
    float4 p[8];
    int pos[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int s = s0 + 4 * k + g;
      pos[k] = -1;
      if (s < ns) {
        const float bd = ws.leaf_lo[s].x;
        const float4 rg = ws.leaf_hi[s];
        if ((variant == 1 || bd <= bnd) && o < f2i(rg.w)) pos[k] = f2i(rg.z) + o;
      }
      p[k] = bv.pts[pos[k] >= 0 ? pos[k] : last];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (pos[k] >= 0) mine.offer(d2_ref(qx, qy, qz, p[k].x, p[k].y, p[k].z), f2i(p[k].w), pos[k]);
  }
  r = wave_lex_min(mine);
  wave_sync();
}

// The staging walk of one query from the sp node ids on ws.stack: up to 64
// nodes tested per round (one coalesced load each, all in flight), internal
// nodes whose box meets the ball push both children, leaves are staged and
// scanned in flushes that tighten the (uniform) bound.  Exact over the
// subtrees on the initial stack.
template <class R>
__device__ __forceinline__ void nn_wave_walk(const BvhView& bv, int sp, float qx, float qy,
                                             float qz, R& r, WnnScratch& ws, int variant = 0) {
  const int lane = __lane_id();
  const int nl = bv.nleaves;
  R mine = r;
  int ns = 0;
  const uint64_t lt = (1ull << lane) - 1ull;
  wave_sync();
  while (sp > 0 || ns > 0) {
    if (sp > 0) {
      const int k = min(min(kWnnPop, sp), max(1, (kWnnStack - 48 - sp) / 2));
      int node = 0;
      if (lane < k) node = ws.stack[sp - 1 - lane];
      sp -= k;
      wave_sync();
      bool pass = false;
      float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
      float bd = 0.f;
      if (lane < k) {
        lo = bv.nodes[2 * node];
        hi = bv.nodes[2 * node + 1];
        bd = box_d2(qx, qy, qz, lo, hi);
        pass = bd <= r.bound();
      }
      const bool isleaf = node >= nl;
      const uint64_t im = __ballot(pass && !isleaf);
      const uint64_t lm = __ballot(pass && isleaf);
      if (pass && !isleaf) {
        const int rk = __popcll(im & lt);
        const int nc = near_child(node, lo, hi, qx, qy, qz);
        ws.stack[sp + 2 * rk] = nc ^ 1;
        ws.stack[sp + 2 * rk + 1] = nc;
      }
      if (pass && isleaf) {
        const int rk = __popcll(lm & lt);
        ws.leaf_lo[ns + rk] = make_float4(bd, 0.f, 0.f, i2f(node - nl));
      }
      sp += 2 * __popcll(im);
      ns += __popcll(lm);
      wave_sync();
    }
    if (ns > kWnnLeaves - kWnnPop || (sp == 0 && ns > 0)) {
      wnn_flush_one(bv, ws, ns, qx, qy, qz, mine, r, variant);
      ns = 0;
    }
  }
}

// r: uniform across the wave (the warm offer, or empty); returns the exact
// answer, uniform.  warm: sorted position to start from (-1: the root).
// The walk starts at the warm leaf and the sibling of every ancestor (a
// partition of the tree).
template <class R>
__device__ __forceinline__ void nn_wave_one(const BvhView& bv, int warm, float qx, float qy,
                                            float qz, R& r, WnnScratch& ws, int variant = 0) {
  const int lane = __lane_id();
  const int nl = bv.nleaves;
  if (bv.m <= 0 || !finite3(qx, qy, qz)) return;
  const unsigned start = (warm >= 0 && warm < bv.m) ? (unsigned)(nl + leaf_of(bv, warm)) : 1u;
  const int depth = 31 - __clz(start);
  if (lane < depth) ws.stack[lane] = (int)((start >> (depth - 1 - lane)) ^ 1u);
  if (lane == 0) ws.stack[depth] = (int)start;
  nn_wave_walk(bv, depth + 1, qx, qy, qz, r, ws, variant);
}

// Exact 1-NN of one query through the level-2 (shift = kAdj2Shift: items =
// nodes of 8 leaves) or level-3 (kAdj3Shift: nodes of 64 leaves) adjacency
// of the warm point's item, whole wave: the same coverage argument as
// rst_bvh.hpp adj2_search / adj3_search, with the 24 entries tested by 24
// lanes at once.  Level 2 stages the candidate nodes' leaves directly (one
// round of box loads); level 3 seeds the staging walk with the candidate
// nodes.  Returns false, having offered nothing, when the ball is not
// covered.  r uniform in and out.
template <class R>
__device__ __forceinline__ bool nn_wave_adj(const BvhView& bv, const AdjView& av, int shift,
                                            int warm, float qx, float qy, float qz, R& r,
                                            WnnScratch& ws) {
  const int lane = __lane_id();
  const int nl = bv.nleaves;
  if (nl < (1 << shift) || warm < 0 || warm >= bv.m || !finite3(qx, qy, qz)) return false;
  const float4* ent = shift == kAdj2Shift ? av.ent2 : av.ent3;
  const float* reach = shift == kAdj2Shift ? av.reach2 : av.reach3;
  const int first = nl >> shift;
  const int N = (nl + leaf_of(bv, warm)) >> shift;
  float4 l = make_float4(0.f, 0.f, 0.f, 0.f), h = l;
  int X = -1;
  if (lane < kAdjK) {
    l = ent[((int64_t)(N - first) * kAdjK + lane) * 2];
    h = ent[((int64_t)(N - first) * kAdjK + lane) * 2 + 1];
    X = f2i(h.w);
  }
  const float4 nlo = bv.nodes[2 * N], nhi = bv.nodes[2 * N + 1];
  const float rch = reach[N - first];
  // margins cover float rounding of every distance (rst_bvh.hpp adj_search)
  const float dl = sqrtf(box_d2(qx, qy, qz, nlo, nhi)) * 1.00001f;
  const float rb = sqrtf(r.bound()) * 1.00001f + 1e-30f;
  if (!(dl + rb < rch * 0.99999f)) return false;
  // entries are sorted by box distance: the early exit of the sequential
  // scan is the same per-entry test
  const bool cand = X >= 0 && !(l.w * 0.99999f - dl > rb) && box_d2(qx, qy, qz, l, h) <= r.bound();
  const uint64_t cm = __ballot(cand);
  const uint64_t lt = (1ull << lane) - 1ull;
  const int nc = __popcll(cm);
  if (cand) ws.stack[__popcll(cm & lt)] = first + X;
  wave_sync();
  if (shift != kAdj2Shift) {
    nn_wave_walk(bv, nc, qx, qy, qz, r, ws);
    return true;
  }
  // level 2: the candidate nodes' 8 leaves each, boxes tested by the wave
  R mine = r;
  int ns = 0;
  const int total = nc << kAdj2Shift;
  for (int i0 = 0; i0 < total; i0 += kWave) {
    const int idx = i0 + lane;
    bool pass = false;
    float bd = 0.f;
    int L = 0;
    if (idx < total) {
      const int node = ws.stack[idx >> kAdj2Shift];
      L = (node << kAdj2Shift) - nl + (idx & ((1 << kAdj2Shift) - 1));
      bd = box_d2(qx, qy, qz, bv.nodes[2 * (nl + L)], bv.nodes[2 * (nl + L) + 1]);
      pass = bd <= r.bound();
    }
    const uint64_t lm = __ballot(pass);
    if (pass) ws.leaf_lo[ns + __popcll(lm & lt)] = make_float4(bd, 0.f, 0.f, i2f(L));
    ns += __popcll(lm);
    wave_sync();
    if (ns > kWnnLeaves - kWave || (i0 + kWave >= total && ns > 0)) {
      wnn_flush_one(bv, ws, ns, qx, qy, qz, mine, r);
      ns = 0;
    }
  }
  return true;
}

}  // namespace rst

namespace rst {

// ---- per-lane search through the leaf adjacency (the ICP fast path) ------------
// rst_bvh.hpp adj_search with every load issued early: adjacency entries
// four at a time (each entry carries its leaf's box, so a test needs no
// further gather) and leaf points eight at a time, unconditionally (index
// clamped), so a lane's dependent chain is warm point -> entries -> points.
template <class R>
RST_HD void scan_range_wide(const BvhView& bv, int b, int n, float qx,
                                                float qy, float qz, R& r) {
  const int last = bv.m - 1;
  for (int j0 = 0; j0 < n; j0 += 8) {
    float4 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = bv.pts[min(b + j0 + j, last)];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j0 + j < n) r.offer(d2_ref(qx, qy, qz, p[j].x, p[j].y, p[j].z), f2i(p[j].w), b + j0 + j);
  }
}

// Best1 form (the ICP fast path): the batch loaded from one base address
// (immediate offsets; kPtsPad covers the overrun), the distance with packed
// (x, y) arithmetic (the roundings of d2_ref: ((dx*dx + dy*dy) + dz*dz), no
// contraction), and lex_less as one unsigned 64-bit compare of (d2 bits,
// id): d2 >= 0 orders like its bits, and NaN / inf keys never beat the
// FLT_MAX start, as with the float compare.
typedef float rst_f2 __attribute__((ext_vector_type(2)));
template <>
RST_HD void scan_range_wide<Best1>(const BvhView& bv, int b, int n, float qx, float qy, float qz,
                                   Best1& r) {
  const rst_f2 qxy = {qx, qy};
  uint64_t best = ((uint64_t)(uint32_t)f2i(r.d) << 32) | (uint32_t)r.id;
  int bj = -1;  // offset in the range of the best point so far (uniform candidates)
  for (int j0 = 0; j0 < n; j0 += 8) {
    const float4* base = bv.pts + b + j0;
    float4 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = base[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const rst_f2 pxy = {p[j].x, p[j].y};
      const rst_f2 dxy = qxy - pxy;
      const rst_f2 sq = dxy * dxy;
      const float dz = qz - p[j].z;
      float d2 = sq.x + sq.y;
      d2 = d2 + dz * dz;
      const uint64_t key = ((uint64_t)(uint32_t)f2i(d2) << 32) | (uint32_t)f2i(p[j].w);
      const bool t = (j0 + j < n) & (key < best);
      best = t ? key : best;
      bj = t ? j0 + j : bj;
    }
  }
  r.d = i2f((int)(uint32_t)(best >> 32));
  r.id = (int)(uint32_t)best;
  r.pos = bj >= 0 ? b + bj : r.pos;
}

// Best2 form: the two lexicographically smallest (d2, id) keys as 64-bit
// integers (d2 >= 0 orders like its bits); a point already held (same id)
// is never re-inserted.
template <>
RST_HD void scan_range_wide<Best2>(const BvhView& bv, int b, int n, float qx, float qy, float qz,
                                   Best2& r) {
  const rst_f2 qxy = {qx, qy};
  uint64_t k0 = ((uint64_t)(uint32_t)f2i(r.d[0]) << 32) | (uint32_t)r.id[0];
  uint64_t k1 = ((uint64_t)(uint32_t)f2i(r.d[1]) << 32) | (uint32_t)r.id[1];
  int p0 = r.pos[0], p1 = r.pos[1];
  for (int j0 = 0; j0 < n; j0 += 8) {
    const float4* base = bv.pts + b + j0;
    float4 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = base[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const rst_f2 pxy = {p[j].x, p[j].y};
      const rst_f2 dxy = qxy - pxy;
      const rst_f2 sq = dxy * dxy;
      const float dz = qz - p[j].z;
      float d2 = sq.x + sq.y;
      d2 = d2 + dz * dz;
      const uint64_t key = ((uint64_t)(uint32_t)f2i(d2) << 32) | (uint32_t)f2i(p[j].w);
      const bool in = (j0 + j < n) & (key != k0) & (key < k1);
      const bool first = in & (key < k0);
      const int pos = b + j0 + j;
      k1 = first ? k0 : (in ? key : k1);
      p1 = first ? p0 : (in ? pos : p1);
      k0 = first ? key : k0;
      p0 = first ? pos : p0;
    }
  }
  r.d[0] = i2f((int)(uint32_t)(k0 >> 32));
  r.id[0] = (int)(uint32_t)k0;
  r.pos[0] = p0;
  r.d[1] = i2f((int)(uint32_t)(k1 >> 32));
  r.id[1] = (int)(uint32_t)k1;
  r.pos[1] = p1;
}

// When the ball is not covered (the query moved away from its last
// neighbour, early ICP iterations), the warm candidate is first walked
// through the adjacency: the listed leaf whose box is nearest to the query
// is scanned and the best point found becomes the new start, up to
// kWalkSteps times.  Walking only lowers the bound; exactness still comes
// from the coverage test of the final leaf.
#ifndef RST_WALK_STEPS
#define RST_WALK_STEPS 1
#endif
constexpr int kWalkSteps = RST_WALK_STEPS;

// sqrt for the coverage / stop tests: the hardware v_sqrt_f32 (about 1 ulp)
// on the device; every use carries the 1.00001 / 0.99999 margins of
// rst_bvh.hpp adj_search, far wider than its error, so the tests stay
// conservative (the correctly rounded sqrtf costs ~15 instructions per call)
RST_HD float margin_sqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sqrtf(x);
#else
  return sqrtf(x);
#endif
}

template <class R>
RST_HD bool adj_search_wide(const BvhView& bv, const AdjView& av, int start,
                                                float qx, float qy, float qz, R& r,
                                                int* walked = nullptr) {
  const int nl = bv.nleaves;
  int L = leaf_of(bv, start);
  float dl;
  for (int step = 0;; ++step) {
    const float4 lo = bv.nodes[2 * (nl + L)], hi = bv.nodes[2 * (nl + L) + 1];
    const float reach = av.reach[L];
    // same margins as rst_bvh.hpp adj_search
    dl = margin_sqrt(box_d2(qx, qy, qz, lo, hi)) * 1.00001f;
    if (dl + margin_sqrt(r.bound()) * 1.00001f + 1e-30f < reach * 0.99999f) break;
    if (walked) *walked = step + 1;
    if (step == kWalkSteps) return false;
    // walk: scan the listed leaf nearest to the query (other than L)
    const float4* e = av.ent + (int64_t)L * kAdjK * 2;
    float bb = FLT_MAX;
    int bx = -1;
    for (int k = 1; k < kAdjK; ++k) {
      const float4 l = e[2 * k], h = e[2 * k + 1];
      const int tag = f2i(h.w);
      const float b = box_d2(qx, qy, qz, l, h);
      const bool t = tag >= 0 && b < bb;
      bb = t ? b : bb;
      bx = t ? tag : bx;
    }
    if (bx < 0 || !(bb < r.d)) return false;
    scan_range_wide(bv, bx >> 5, bx & 31, qx, qy, qz, r);
    L = leaf_of(bv, r.pos);
  }
  const float4* e = av.ent + (int64_t)L * kAdjK * 2;
  for (int k0 = 0; k0 < kAdjK; k0 += 4) {
    float4 l[4], h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      l[j] = e[2 * (k0 + j)];
      h[j] = e[2 * (k0 + j) + 1];
    }
    bool stop = false;
    // the batch's stop radius from the bound at its start: the bound only
    // shrinks, so a later entry tested against it stops no earlier (exact)
    const float rad = margin_sqrt(r.bound()) * 1.00001f + 1e-30f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (stop) break;
      const int tag = f2i(h[j].w);
      if (tag < 0 || l[j].w * 0.99999f - dl > rad) {
        stop = true;
      } else if (box_d2(qx, qy, qz, l[j], h[j]) <= r.bound()) {
        scan_range_wide(bv, tag >> 5, tag & 31, qx, qy, qz, r);
      }
    }
    if (stop) break;
  }
  return true;
}

// The certificate search of the ICP fast path (icp.hip k_icp_nn): the two
// nearest through the leaf adjacency of the leaf holding sorted position
// `start`, every listed leaf whose box meets the ball of the running SECOND
// distance scanned.  Returns the covered radius Rc (reach - dist(q, box(L)),
// float margins applied): every point within Rc of q lies in a listed leaf.
// Hence, with the scan's stop rule at the second radius r2:
//   * r.first() is the exact nearest neighbour when sqrt(d[0]) < Rc;
//   * every point other than it lies at >= min(r2, Rc) from q -- the
//     point's certificate for later iterations (a query that moved by
//     delta keeps the neighbour while |q' - p| + delta < that bound).
// r arrives holding the warm offers.  Like adj_search_wide, one walk step
// moves L to the listed leaf nearest to q when q lies outside the coverage
// of the start leaf.
RST_HD float adj_search2(const BvhView& bv, const AdjView& av, int start, float qx, float qy,
                         float qz, Best2& r) {
  const int nl = bv.nleaves;
  int L = leaf_of(bv, start);
  float dl = 0.f, reach = 0.f;
  for (int step = 0;; ++step) {
    const float4 lo = bv.nodes[2 * (nl + L)], hi = bv.nodes[2 * (nl + L) + 1];
    reach = av.reach[L];
    dl = margin_sqrt(box_d2(qx, qy, qz, lo, hi)) * 1.00001f;
    if (dl + margin_sqrt(r.d[0]) * 1.00001f + 1e-30f < reach * 0.99999f || step == kWalkSteps)
      break;
    const float4* e = av.ent + (int64_t)L * kAdjK * 2;
    float bb = FLT_MAX;
    int bx = -1;
    for (int k = 1; k < kAdjK; ++k) {
      const float4 l = e[2 * k], h = e[2 * k + 1];
      const int tag = f2i(h.w);
      const float b = box_d2(qx, qy, qz, l, h);
      const bool t = tag >= 0 && b < bb;
      bb = t ? b : bb;
      bx = t ? tag : bx;
    }
    if (bx < 0 || !(bb < r.d[0])) break;
    scan_range_wide(bv, bx >> 5, bx & 31, qx, qy, qz, r);
    L = leaf_of(bv, r.pos[0]);
  }
  const float rc = reach * 0.99999f - dl;
  if (!(dl + margin_sqrt(r.d[0]) * 1.00001f + 1e-30f < reach * 0.99999f)) return rc;
  const float4* e = av.ent + (int64_t)L * kAdjK * 2;
  for (int k0 = 0; k0 < kAdjK; k0 += 4) {
    float4 l[4], h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      l[j] = e[2 * (k0 + j)];
      h[j] = e[2 * (k0 + j) + 1];
    }
    bool stop = false;
    // stop radius from the second bound at the batch's start (it only
    // shrinks: a later entry tested against it stops no earlier)
    const float rad = margin_sqrt(r.d[1]) * 1.00001f + 1e-30f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (stop) break;
      const int tag = f2i(h[j].w);
      if (tag < 0 || l[j].w * 0.99999f - dl > rad) {
        stop = true;
      } else if (box_d2(qx, qy, qz, l[j], h[j]) <= r.d[1]) {
        scan_range_wide(bv, tag >> 5, tag & 31, qx, qy, qz, r);
      }
    }
    if (stop) break;
  }
  return rc;
}

// The two nearest of one query through the leaf adjacency of the leaf
// holding sorted position `warm`, whole wave (adj_search2 with the 24
// entries tested by 24 lanes at once and the listed leaves' points scanned
// 16 lanes per leaf, all loads of a round in flight): a few memory
// latencies instead of a lane's chain of one per leaf.  r (uniform) holds
// the seeds.  Returns the covered radius Rc as adj_search2 does -- r.first()
// is exact when sqrt(d[0]) < Rc, and min(r2, Rc) bounds every other point;
// when the warm leaf's coverage does not reach the first radius nothing is
// scanned (the return value then fails that test).
template <class R>
__device__ __forceinline__ float nn_wave_adj1(const BvhView& bv, const AdjView& av, int warm,
                                              float qx, float qy, float qz, R& r, WnnScratch& ws) {
  const int lane = __lane_id();
  const int nl = bv.nleaves;
  const int L = leaf_of(bv, warm);
  float4 l = make_float4(0.f, 0.f, 0.f, 0.f), h = l;
  int tag = -1;
  if (lane < kAdjK) {
    l = av.ent[((int64_t)L * kAdjK + lane) * 2];
    h = av.ent[((int64_t)L * kAdjK + lane) * 2 + 1];
    tag = f2i(h.w);
  }
  const float4 nlo = bv.nodes[2 * (nl + L)], nhi = bv.nodes[2 * (nl + L) + 1];
  const float reach = av.reach[L];
  // the margins of adj_search2
  const float dl = margin_sqrt(box_d2(qx, qy, qz, nlo, nhi)) * 1.00001f;
  const float rc = reach * 0.99999f - dl;
  if (!(dl + margin_sqrt(r.d[0]) * 1.00001f + 1e-30f < reach * 0.99999f)) return rc;
  // entries are sorted by bbd: testing each against the stop rule is the
  // sequential scan's early exit
  const float rad = margin_sqrt(r.bound()) * 1.00001f + 1e-30f;
  const float bd = box_d2(qx, qy, qz, l, h);
  const bool cand = tag >= 0 && !(l.w * 0.99999f - dl > rad) && bd <= r.bound();
  const uint64_t cm = __ballot(cand);
  const int ns = __popcll(cm);
  if (cand) {
    const int k = __popcll(cm & ((1ull << lane) - 1ull));
    ws.leaf_lo[k] = make_float4(bd, 0.f, 0.f, 0.f);
    ws.leaf_hi[k] = make_float4(0.f, 0.f, i2f(tag >> 5), i2f(tag & 31));
  }
  wave_sync();
  R mine = r;
  if (ns > 0) wnn_scan_ranges(bv, ws, ns, qx, qy, qz, mine, r, 0);
  return rc;
}

// adj_search2 with one query per row of 16 lanes (lanes 16g .. 16g+15 hold the same query q and the same seeds r), four
// queries per wavefront.  The warm leaf's 24 adjacency entries are tested
// by the row at once (lane k: entries k and k + 16), the candidates' point
// ranges compacted in LDS (`tags`, 24 ints per row), and each lane takes
// one point of every candidate leaf (a leaf holds <= 16), all loads in
// flight before the offers; a row merge then leaves every lane of the row
// with the row's two nearest.  Candidates are tested against the seeds'
// second bound (the sequential scan tightens it as it goes: this tests a
// superset).  Returns the covered radius Rc exactly as adj_search2: r.first()
// is exact when sqrt(d[0]) < Rc, min(r2, Rc) bounds every other point.
// Rows with act == false take no part in the loads (their result is
// meaningless); the whole wavefront must call it.
__device__ __forceinline__ float row_adj2(const BvhView& bv, const AdjView& av, bool act, int warm,
                                          float qx, float qy, float qz, Best2& r, int* tags) {
  const int lane = __lane_id();
  const int sub = lane & 15;
  const int nl = bv.nleaves;
  const int L = act ? leaf_of(bv, warm) : 0;
  float4 l0 = make_float4(0.f, 0.f, 0.f, 0.f), h0 = l0, l1 = l0, h1 = l0;
  int t0 = -1, t1 = -1;
  if (act) {
    const float4* e = av.ent + (int64_t)L * kAdjK * 2;
    l0 = e[2 * sub];
    h0 = e[2 * sub + 1];
    t0 = f2i(h0.w);
    if (sub < kAdjK - 16) {
      l1 = e[2 * (sub + 16)];
      h1 = e[2 * (sub + 16) + 1];
      t1 = f2i(h1.w);
    }
  }
  float4 nlo = l0, nhi = l0;
  float reach = 0.f;
  if (act) {
    nlo = bv.nodes[2 * (nl + L)];
    nhi = bv.nodes[2 * (nl + L) + 1];
    reach = av.reach[L];
  }
  // the margins of adj_search2
  const float dl = margin_sqrt(box_d2(qx, qy, qz, nlo, nhi)) * 1.00001f;
  const float rc = reach * 0.99999f - dl;
  const bool cov = act && dl + margin_sqrt(r.d[0]) * 1.00001f + 1e-30f < reach * 0.99999f;
  const float rad = margin_sqrt(r.d[1]) * 1.00001f + 1e-30f;
  const bool c0 = cov && t0 >= 0 && !(l0.w * 0.99999f - dl > rad) && box_d2(qx, qy, qz, l0, h0) <= r.d[1];
  const bool c1 = cov && t1 >= 0 && !(l1.w * 0.99999f - dl > rad) && box_d2(qx, qy, qz, l1, h1) <= r.d[1];
  const int sh = lane & ~15;
  const uint32_t m0 = (uint32_t)(__ballot(c0) >> sh) & 0xffffu;
  const uint32_t m1 = (uint32_t)(__ballot(c1) >> sh) & 0xffffu;
  const uint32_t below = (1u << sub) - 1u;
  if (c0) tags[__popc(m0 & below)] = t0;
  if (c1) tags[__popc(m0) + __popc(m1 & below)] = t1;
  wave_sync();
  const int nc = __popc(m0) + __popc(m1);
  Best2 mine = r;
  const int last = bv.m - 1;
  for (int c0i = 0; c0i < nc; c0i += 8) {
    float4 p[8];
    int pos[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pos[k] = -1;
      if (c0i + k < nc) {
        const int tg = tags[c0i + k];
        if (sub < (tg & 31)) pos[k] = (tg >> 5) + sub;
      }
      p[k] = bv.pts[pos[k] >= 0 ? pos[k] : last];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (pos[k] >= 0) mine.offer(d2_ref(qx, qy, qz, p[k].x, p[k].y, p[k].z), f2i(p[k].w), pos[k]);
  }
  r = wave_lex_min<8>(mine);
  wave_sync();
  return rc;
}

// The certificate bound of adj_search2's result (0: none): min(r2, Rc)
// with the 1e-5 relative margins of every distance test here.
RST_HD float cert_bound(const Best2& r, float rc) {
  const float r2 = r.d[1] < FLT_MAX ? margin_sqrt(r.d[1]) * 0.99999f : FLT_MAX;
  const float g = fminf(r2, rc);
  return g > 0.f ? g : 0.f;
}

__device__ __forceinline__ bool box_meets(const float4& lo, const float4& hi, float lx, float ly,
                                          float lz, float hx, float hy, float hz) {
  return lo.x <= hx && hi.x >= lx && lo.y <= hy && hi.y >= ly && lo.z <= hz && hi.z >= lz;
}

// ---- ball tiles: the cold iterations' wave-shared search --------------------------------
// The 64 queries of a wavefront (Morton-consecutive: one compact patch) each
// hold an upper bound u_i of their nearest distance (the distance to a seed
// point: the last neighbour, or the Morton seed).  The wave walks the BVH
// top-down once for the box B = union of the balls (q_i, u_i) (64 nodes per
// round, the stack in LDS), streaming the leaves that meet B through LDS
// kBallChunk points at a time; every lane scans every chunk (broadcast
// reads) for its two nearest, and after each chunk the balls -- and B --
// shrink to the lanes' new first distances (branch and bound for the whole
// wave).  A node is dropped only when it misses the current B, which holds
// every later B, so every target point inside the final B is scanned: each
// distance Mq from q_i to the outside of the final B bounds every unscanned
// point: the lane's first is exact when it lies within Mq (always, unless
// the RST_BALL_CAP cap kept its ball out of B), and min(r2, Mq) is its
// certificate.  Returns false (lanes keep a
// valid but unfinished r) when the walk exceeds kBallMaxChunks chunks: the
// caller finishes those lanes alone.
constexpr int kBallChunk = 512;    // staged points per scan (a loop's own choice: BallScratchT)
constexpr int kBallLeaves = 128;   // collected leaves (a round adds <= 64)
constexpr int kBallStack = 320;    // node ids
#ifndef RST_BALL_MAX_CHUNKS
#define RST_BALL_MAX_CHUNKS 48
#endif
constexpr int kBallMaxChunks = RST_BALL_MAX_CHUNKS;
template <int C>
struct BallScratchT {              // per-wave LDS (~12.5 KB at C = 512)
  static constexpr int kChunk = C;
  float4 pts[C];                   // x, y, z, original index bits
  int pos[C];                      // sorted position
  int stack[kBallStack];
  int leaves[kBallLeaves];
};
using BallScratch = BallScratchT<kBallChunk>;

__device__ __forceinline__ float wave_min_f(float x) { return bfly_reduce<6>(x, OpMinF{}); }
__device__ __forceinline__ float wave_max_f(float x) { return bfly_reduce<6>(x, OpMaxF{}); }

// The box of the active lanes' balls (radius: the first distance, rounded
// up by the 1e-5 margins of every coverage test here, capped at
// RST_BALL_CAP metres: a lane whose ball the box does not hold is answered
// only if its first ends up inside the box -- the caller checks -- so the
// cap bounds the work, never the exactness).
#ifndef RST_BALL_CAP
#define RST_BALL_CAP 0.10f  // r02z2: 0.10 m / 48 chunks 13.90 ms per pair, uncapped / 24 14.06
#endif
__device__ __forceinline__ void ball_box(bool act, float qx, float qy, float qz, const Best2& r,
                                         float4& lo, float4& hi) {
  // (+4 um: the box corners q -/+ u round to float at up to ~1 ulp of the
  // coordinates, < 4 um for |q| < 32 m)
  const float u = act ? fminf(margin_sqrt(r.d[0]) * 1.00001f + 4e-6f, RST_BALL_CAP) : 0.f;
  lo.x = wave_min_f(act ? qx - u : FLT_MAX);
  lo.y = wave_min_f(act ? qy - u : FLT_MAX);
  lo.z = wave_min_f(act ? qz - u : FLT_MAX);
  hi.x = wave_max_f(act ? qx + u : -FLT_MAX);
  hi.y = wave_max_f(act ? qy + u : -FLT_MAX);
  hi.z = wave_max_f(act ? qz + u : -FLT_MAX);
}

// Scan the leaves ts.leaves[0, nlv) for every lane: their points staged
// kBallChunk at a time, 16 lanes per leaf.  Returns the chunk count, or -1
// when an index guard trips (never expected).
template <class TS>
__device__ __forceinline__ int ball_flush(const BvhView& bv, TS& ts, int nlv, float qx,
                                          float qy, float qz, Best2& r, int4& det) {
  const int lane = __lane_id();
  int chunks = 0;
  for (int l0 = 0; l0 < nlv;) {
    // leaves [l0, l1) fill one chunk (<= 16 points each)
    const int l1 = min(nlv, l0 + TS::kChunk / 16);
    int b = 0, c = 0;
    bool bad = false;
    if (lane < l1 - l0) {
      const int L = ts.leaves[l0 + lane];
      bad = (uint32_t)L >= (uint32_t)bv.nleaves;
      if (!bad) {
        b = leaf_begin(bv, L);
        c = leaf_begin(bv, L + 1) - b;
        bad = c < 0 || c > 16 || b < 0 || b + c > bv.m;
      }
    }
    const uint64_t bm = __ballot(bad);
    if (bm != 0) {
      const int j = __ffsll((long long)bm) - 1;
      det = make_int4(__shfl(l0 + lane < nlv ? ts.leaves[l0 + lane] : -7, j, kWave),
                      __shfl(b, j, kWave), __shfl(c, j, kWave), nlv * 1000 + l0);
      return -1;
    }
    int inc = c;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int y = __shfl_up(inc, o, kWave);
      if (lane >= o) inc += y;
    }
    const int total = __builtin_amdgcn_readlane(inc, kWave - 1);
    const int off = inc - c;
    const int g = lane >> 4, o = lane & 15;
    for (int k0 = 0; k0 < l1 - l0; k0 += 4) {  // one leaf per 16 lanes
      const int kk = k0 + g;
      const int lb = __shfl(b, kk & 63, kWave), lc = __shfl(c, kk & 63, kWave);
      const int lo = __shfl(off, kk & 63, kWave);
      if (kk < l1 - l0 && o < lc) {
        ts.pts[lo + o] = bv.pts[lb + o];
        ts.pos[lo + o] = lb + o;
      }
    }
    wave_sync();
    {
      uint64_t k0 = ((uint64_t)(uint32_t)f2i(r.d[0]) << 32) | (uint32_t)r.id[0];
      uint64_t k1 = ((uint64_t)(uint32_t)f2i(r.d[1]) << 32) | (uint32_t)r.id[1];
      int j0 = -1, j1 = -1;
      for (int j = 0; j < total; ++j) {
        const float4 p = ts.pts[j];
        const float d2 = d2_ref(qx, qy, qz, p.x, p.y, p.z);
        const uint64_t key = ((uint64_t)(uint32_t)f2i(d2) << 32) | (uint32_t)f2i(p.w);
        const bool in = (key != k0) & (key < k1);
        const bool first = in & (key < k0);
        k1 = first ? k0 : (in ? key : k1);
        j1 = first ? j0 : (in ? j : j1);
        k0 = first ? key : k0;
        j0 = first ? j : j0;
      }
      // positions of the chunk's winners before the next chunk overwrites it
      const int p0 = j0 >= 0 ? ts.pos[j0] : r.pos[0];
      const int p1 = j1 >= 0 ? ts.pos[j1] : (j0 >= 0 ? r.pos[0] : r.pos[1]);
      if (j0 >= 0 || j1 >= 0) {
        r.d[0] = i2f((int)(uint32_t)(k0 >> 32));
        r.id[0] = (int)(uint32_t)k0;
        r.d[1] = i2f((int)(uint32_t)(k1 >> 32));
        r.id[1] = (int)(uint32_t)k1;
        r.pos[1] = p1;
        r.pos[0] = p0;
      }
    }
    wave_sync();
    l0 = l1;
    ++chunks;
  }
  return chunks;
}

// act: the lane holds a query (r: its seeds, r.d[0] finite); inactive lanes
// only help.  On true, Mq (per active lane) = the distance from q to the
// outside of the final box, margins applied: the lane's first is exact when
// it lies within Mq (every point inside the box was scanned).  The whole
// wave calls it.
template <class TS>
__device__ __forceinline__ bool ball_tile_search(const BvhView& bv, bool act, float qx, float qy,
                                                 float qz, Best2& r, float& mq, TS& ts,
                                                 int& gfail, int4& det, int& chunks) {
  constexpr int kMaxChunks = kBallMaxChunks * kBallChunk / TS::kChunk;  // (the same staged points)
  const int lane = __lane_id();
  const int nl = bv.nleaves;
  const uint64_t lt = (1ull << lane) - 1ull;
  float4 lo, hi;
  ball_box(act, qx, qy, qz, r, lo, hi);
  if (lane == 0) ts.stack[0] = 1;
  int sp = 1, nlv = 0;
  chunks = 0;
  wave_sync();
  while (sp > 0 || nlv > 0) {
    if (sp > 0 && nlv <= kBallLeaves - kWave && sp <= kBallStack - 2 * kWave) {
      const int k = min(kWave, sp);
      int node = 0;
      if (lane < k) node = ts.stack[sp - 1 - lane];
      sp -= k;
      wave_sync();
      bool pass = false;
      const uint64_t gm = __ballot(lane < k && (node < 1 || node >= 2 * nl));
      if (gm != 0) {  // index guard
        const int j = __ffsll((long long)gm) - 1;
        det = make_int4(__shfl(node, j, kWave), sp, nlv, nl);
        gfail = 1;
        return false;
      }
      if (lane < k) {
        const float4 nlo = bv.nodes[2 * node], nhi = bv.nodes[2 * node + 1];
        pass = box_meets(nlo, nhi, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z);
      }
      const bool isleaf = node >= nl;
      const uint64_t im = __ballot(pass && !isleaf), lm = __ballot(pass && isleaf);
      if (pass && !isleaf) {
        const int rk = __popcll(im & lt);
        ts.stack[sp + 2 * rk] = 2 * node;
        ts.stack[sp + 2 * rk + 1] = 2 * node + 1;
      }
      if (pass && isleaf) ts.leaves[nlv + __popcll(lm & lt)] = node - nl;
      sp += 2 * __popcll(im);
      nlv += __popcll(lm);
      wave_sync();
      if (sp > 0 && nlv <= kBallLeaves - kWave && sp <= kBallStack - 2 * kWave) continue;
    }
    if (nlv == 0) {
      if (sp == 0) break;
      return false;  // stack full with no leaf to drain (never expected)
    }
    const int c = ball_flush(bv, ts, nlv, qx, qy, qz, r, det);
    if (c < 0) {
      gfail = 2;
      return false;
    }
    chunks += c;
    nlv = 0;
    if (chunks > kMaxChunks) return false;
    ball_box(act, qx, qy, qz, r, lo, hi);  // the balls shrink
  }
  const float m = fminf(fminf(fminf(qx - lo.x, hi.x - qx), fminf(qy - lo.y, hi.y - qy)),
                        fminf(qz - lo.z, hi.z - qz));
  mq = m * 0.99999f;
  return true;
}

// ---- pixel tiles: exact searches through a frame target's pixel grid -------------------
// A frame target's points come from its depth image (unproject.hip): point
// (a, b) of the level grid (stride s) lies on the ray of full-resolution
// pixel (a s, b s), P = z ((u - cx) / fx, (v - cy) / fy, 1), so
// fx P.x / P.z + cx = u up to the float roundings of the unprojection
// (relative 2e-7: < 3e-4 px).  For a query q with q.z > r, every x with
// |x - q| <= r projects within
//     |u_x - u_q| <= |fx| r sqrt(q.x^2 + q.z^2) / (q.z (q.z - r))
// of q's projection u_q (the difference of ratios x.x / x.z - q.x / q.z has
// numerator q.z d.x - q.x d.z <= r |(q.z, q.x)| and denominator
// q.z x.z >= q.z (q.z - r)), likewise v with fy, q.y.  So the points of that
// pixel window are every target point within r of q: a lane that scans the
// window of a radius r at least the distance of some target point (its
// seed) has its exact nearest, and min(second, r) is its certificate.  The
// window is padded by 0.1 % and 0.02 px (the float arithmetic of the bound
// and the projection).  The wave stages the union of its lanes' windows in
// LDS, row-major, PixScratch<CH>::kN pixels at a time (PixView::pts and
// map, one load each per pixel, all in flight), and each lane scans its own
// window from LDS.  Lanes whose window exceeds RST_PIX_MAX_HALF pixels, or
// whose query lies within 2 r of the camera plane, and waves whose union
// exceeds kPixMaxW x 8 chunks, are left to the BVH searches (false).
#ifndef RST_PIX_MAX_HALF
#define RST_PIX_MAX_HALF 24.0f  // half-width cap of a lane's window (level pixels; r02: 6 -> 24.4k it/s, 8 -> 23.6k, 4 -> 22.9k; r11, the batched REF loop's k_icp_fb rows: 6 31.0k, 10 31.2k, 16 31.5k, 24 31.6k, 32 31.5k)
#endif
#ifndef RST_RESEED_RING
#define RST_RESEED_RING 0  // > 0: pix_seed_d2 also samples a (2R+1)^2 ring (below)
#endif
#ifndef RST_RESEED_STRIDE
#define RST_RESEED_STRIDE 3
#endif
#ifndef RST_PIX_MIN_PX
#define RST_PIX_MIN_PX 1.5f  // smallest window half-width: the certificate radius
#endif
constexpr int kPixMaxW = 64;

template <int N>
struct PixScratch {  // per-wave LDS: the staged pixels' points
  static constexpr int kN = N;
  float4 pts[N];
};

// A window scan ranks candidates by (d2, original index) -- a frame's
// original indices ascend with its pixels, and each staged pixel carries its
// own (.w) -- and the winner's sorted position comes from the target's
// inverse map once per lane afterwards: one 16-byte load per staged pixel.
constexpr int kPosPending = 0;  // a candidate's position before pix_resolve
__device__ __forceinline__ void pix_resolve(const BvhView& bv, const PixView& pv, Best2& r) {
  if (r.pos[0] >= 0) r.pos[0] = (uint32_t)r.id[0] < (uint32_t)bv.m ? pv.inv[r.id[0]] : -1;
  if (r.pos[1] >= 0) r.pos[1] = (uint32_t)r.id[1] < (uint32_t)bv.m ? pv.inv[r.id[1]] : -1;
}

__device__ __forceinline__ int wave_min_i(int x) { return bfly_reduce<6>(x, OpMinI{}); }
__device__ __forceinline__ int wave_max_i(int x) { return bfly_reduce<6>(x, OpMaxI{}); }

// The pixel window of the ball (q, r), r = max(the seed distance sqrt(d0)
// with margins, RST_PIX_MIN_PX level pixels): false when it is too large
// (or q too near the camera plane); rc = r.
__device__ __forceinline__ bool pix_window(const PixView& pv, float qx, float qy, float qz,
                                           float d0, float maxh, int& a0, int& a1, int& b0,
                                           int& b1, float& rc) {
  if (!(d0 < FLT_MAX) || !(qz > 0.f)) return false;
  const float s = (float)pv.s;
  const float afx = fabsf(pv.fx), afy = fabsf(pv.fy);
  const float rw = fmaxf(margin_sqrt(d0) * 1.00001f + 4e-6f,
                         RST_PIX_MIN_PX * s * qz / fminf(afx, afy));
  if (!(qz > 2.0f * rw)) return false;
  const float iz = 1.0f / qz;
  const float uq = (pv.fx * qx * iz + pv.cx) / s, vq = (pv.fy * qy * iz + pv.cy) / s;
  const float k = rw / (qz * (qz - rw)) / s;
  const float bx = afx * k * sqrtf(qx * qx + qz * qz) * 1.001f + 0.02f;
  const float by = afy * k * sqrtf(qy * qy + qz * qz) * 1.001f + 0.02f;
  if (!(bx <= maxh && by <= maxh && fabsf(uq) < 1e6f && fabsf(vq) < 1e6f)) return false;
  a0 = max(0, (int)ceilf(uq - bx));
  a1 = min(pv.w - 1, (int)floorf(uq + bx));
  b0 = max(0, (int)ceilf(vq - by));
  b1 = min(pv.h - 1, (int)floorf(vq + by));
  rc = rw;
  return a0 <= a1 && b0 <= b1;  // (empty: the seed is off the grid -- never expected)
}

// The smallest squared distance from q to the points of the 3 x 3 pixels
// around its projection (a seed for pix_window; FLT_MAX when none).
__device__ __forceinline__ float pix_seed_d2(const PixView& pv, float qx, float qy, float qz) {
  if (!(qz > 0.f)) return FLT_MAX;
  const float iz = 1.0f / qz;
  const float u = (pv.fx * qx * iz + pv.cx) / (float)pv.s;
  const float v = (pv.fy * qy * iz + pv.cy) / (float)pv.s;
  if (!(u > -2.f && v > -2.f && u < (float)pv.w + 1.f && v < (float)pv.h + 1.f)) return FLT_MAX;
  const int uc = (int)floorf(u + 0.5f), vc = (int)floorf(v + 0.5f);
  float4 p[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {  // all loads first: one latency
    const int uu = uc + k % 3 - 1, vv = vc + k / 3 - 1;
    const bool in = uu >= 0 && vv >= 0 && uu < pv.w && vv < pv.h;
    p[k] = in ? pv.pts[(int64_t)vv * pv.w + uu] : make_float4(NAN, NAN, NAN, 0.f);
  }
  float d = FLT_MAX;
#pragma unroll
  for (int k = 0; k < 9; ++k) d = fminf(d, d2_ref(qx, qy, qz, p[k].x, p[k].y, p[k].z));  // NaN: skipped
#if RST_RESEED_RING
  // a sparse ring of samples RST_RESEED_STRIDE pixels apart out to
  // RST_RESEED_RING strides (the pose moved by centimetres: the point's
  // surface is a few pixels off its projection)
  constexpr int R = RST_RESEED_RING, S = RST_RESEED_STRIDE, D = 2 * R + 1;
  for (int row = 0; row < D; ++row) {
    const int vv = vc + (row - R) * S;
    if (vv < 0 || vv >= pv.h) continue;
    float4 t[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int uu = uc + (k - R) * S;
      t[k] = (uu >= 0 && uu < pv.w) ? pv.pts[(int64_t)vv * pv.w + uu] : make_float4(NAN, NAN, NAN, 0.f);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) d = fminf(d, d2_ref(qx, qy, qz, t[k].x, t[k].y, t[k].z));
  }
#endif
  return d;
}

// Min / max over the 16 lanes of a row, every lane the result, by DPP (no
// LDS trip: a ds_bpermute chain costs each step an LDS round trip, and in
// the window searches' setup four such reductions ran back to back): quad
// butterflies, then row_half_mirror (l <-> 7 - l) and row_mirror
// (l <-> 15 - l) join the quads and the half rows.  The whole wave must be
// active (every caller's is).
__device__ __forceinline__ int row_min_dpp(int x) { return bfly_reduce<4>(x, OpMinI{}); }
__device__ __forceinline__ int row_max_dpp(int x) { return bfly_reduce<4>(x, OpMaxI{}); }
// row r's value (uniform within each row) at lane 16 r, as a scalar
__device__ __forceinline__ int row_val(int x, int r) { return __builtin_amdgcn_readlane(x, 16 * r); }

__device__ __forceinline__ int row_min_i(int x) { return bfly_reduce<4>(x, OpMinI{}); }
__device__ __forceinline__ int row_max_i(int x) { return bfly_reduce<4>(x, OpMaxI{}); }

// act: the lane holds a finite query and d0 = the squared distance of some
// target point (its seed).  On true, r (empty on entry) holds the lane's
// exact two nearest within rc, the first's point in q0, and rc the covered
// radius.  The staged pixels are the union box of the wave's windows, or,
// when that is larger, the four union boxes of its rows of 16 lanes (a
// wave whose queries straddle a jump of the Morton order), laid out one
// after the other; a wave needing more than MaxChunks chunks leaves its
// lanes (false).  The whole wave calls it.
template <int N, int MaxChunks, bool Resolve = true>
__device__ __forceinline__ bool pix_tile_search(const BvhView& bv, const PixView& pv, bool act,
                                                float qx, float qy, float qz, float d0, Best2& r,
                                                float4& q0, PixScratch<N>& ts, float& rc,
                                                float maxh = RST_PIX_MAX_HALF, uint64_t* pclk = nullptr) {
  // (pclk: diagnostics builds' phase clocks -- boxes set up, first chunk
  // staged, scans done; tools/nn_clock.py.  r20: the scans as one flat run
  // of each lane's window pixels, 4 / 6 / 8 LDS reads in flight, measured
  // slower than these rows: k_icp_nn_b 261 -> 273 / 273 / 281 us)
  constexpr int kPer = N / kWave;
  const int lane = __lane_id();
  int a0 = 0, a1 = -1, b0 = 0, b1 = -1;
  rc = 0.f;
  const bool ok = act && pix_window(pv, qx, qy, qz, d0, maxh, a0, a1, b0, b1, rc);
  if (__ballot(ok) == 0) return false;
  // the row boxes (DPP, every lane of a row alike), then the wave box from
  // the four rows' values (readlane: scalars)
  int gA0 = row_min_dpp(ok ? a0 : INT_MAX), gA1 = row_max_dpp(ok ? a1 : INT_MIN);
  int gB0 = row_min_dpp(ok ? b0 : INT_MAX), gB1 = row_max_dpp(ok ? b1 : INT_MIN);
  const bool gok = gA0 <= gA1;  // the row has a window
  const int A0 = min(min(row_val(gA0, 0), row_val(gA0, 1)), min(row_val(gA0, 2), row_val(gA0, 3)));
  const int A1 = max(max(row_val(gA1, 0), row_val(gA1, 1)), max(row_val(gA1, 2), row_val(gA1, 3)));
  const int B0 = min(min(row_val(gB0, 0), row_val(gB0, 1)), min(row_val(gB0, 2), row_val(gB0, 3)));
  const int B1 = max(max(row_val(gB1, 0), row_val(gB1, 1)), max(row_val(gB1, 2), row_val(gB1, 3)));
  if (!gok) gA0 = gA1 = gB0 = gB1 = 0;  // (an empty row box: area 0, never staged)
  const int garea = gok ? (gA1 - gA0 + 1) * (gB1 - gB0 + 1) : 0;
  const int gw = gok ? gA1 - gA0 + 1 : 0;
  // (rows' lanes agree: sum / max over rows 0..3)
  const int gsum = (row_val(garea, 0) + row_val(garea, 1)) + (row_val(garea, 2) + row_val(garea, 3));
  const int gmaxw = max(max(row_val(gw, 0), row_val(gw, 1)), max(row_val(gw, 2), row_val(gw, 3)));
  const int warea = (A1 - A0 + 1) * (B1 - B0 + 1);
  const bool rows4 = gsum < warea;  // uniform
  if (!rows4) {
    gA0 = A0;
    gA1 = A1;
    gB0 = B0;
    gB1 = B1;
  }
  const int total = rows4 ? gsum : warea;
  if ((rows4 ? gmaxw : A1 - A0 + 1) > kPixMaxW || total > N * MaxChunks) return false;
  // box g: origin (bx[g], by[g]), width bw[g], first staged index off[g]
  int bx[4], by[4], bw[4], off[5];
  off[0] = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bx[g] = row_val(gA0, g);
    by[g] = row_val(gB0, g);
    bw[g] = max(row_val(gA1, g) - bx[g] + 1, 1);
    const int ar = rows4 ? row_val(garea, g) : (g == 0 ? warea : 0);
    off[g + 1] = off[g] + ar;
  }
  const int mg = rows4 ? lane >> 4 : 0;  // my box
  const int mx = gA0, my = gB0, mw = max(gA1 - gA0 + 1, 1);
  int moff = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) moff = g == mg ? off[g] : moff;
  if (pclk) pclk[0] = __builtin_amdgcn_s_memtime();
  for (int c0 = 0; c0 < total; c0 += N) {
    const int cnt = min(N, total - c0);
    float4 pp[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {  // every load of the chunk in flight
      const int k = lane + j * kWave;
      pp[j] = make_float4(NAN, NAN, NAN, 0.f);
      if (k < cnt) {
        const int f = c0 + k;
        int g = 0;
#pragma unroll
        for (int h = 1; h < 4; ++h) g = f >= off[h] ? h : g;
        int ox = bx[0], oy = by[0], ow = bw[0], oo = off[0];
#pragma unroll
        for (int h = 1; h < 4; ++h) {
          ox = g == h ? bx[h] : ox;
          oy = g == h ? by[h] : oy;
          ow = g == h ? bw[h] : ow;
          oo = g == h ? off[h] : oo;
        }
        const int kk = f - oo;
        const int rr = (int)(((float)kk + 0.5f) / (float)ow);  // kk / ow (exact: < 2^12)
        const int64_t px = (int64_t)(oy + rr) * pv.w + (ox + kk - rr * ow);
        pp[j] = pv.pts[px];
      }
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int k = lane + j * kWave;
      if (k < cnt) ts.pts[k] = pp[j];
    }
    wave_sync();
    if (pclk && c0 == 0) pclk[1] = __builtin_amdgcn_s_memtime();
    if (ok) {
      // four pixels' LDS reads in flight at a time (a dependent read per
      // pixel would leave the scan bound by LDS latency); an invalid pixel
      // is NaN, so its distance fails every test.  Only the window's rows
      // that meet this chunk: the staged index of (a, b) is
      // moff + (b - my) mw + (a - mx)
      const int lo = c0 - moff + mx - a1, hi = c0 + cnt - 1 - moff + mx - a0;
      const int rb0 = max(b0, my + (lo <= 0 ? -((-lo) / mw) : (lo + mw - 1) / mw));
      const int rb1 = min(b1, my + (hi >= 0 ? hi / mw : -((-hi + mw - 1) / mw)));
      for (int b = rb0; b <= rb1; ++b) {
        const int row = moff + (b - my) * mw - mx - c0;
        for (int a = a0; a <= a1; a += 4) {
          float4 t[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int k = row + a + j;
            const bool in = a + j <= a1 && (uint32_t)k < (uint32_t)cnt;
            t[j] = in ? ts.pts[k] : make_float4(NAN, NAN, NAN, 0.f);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = d2_ref(qx, qy, qz, t[j].x, t[j].y, t[j].z);
            if (d <= r.d[1]) {  // (offer's own test, hoisted; NaN: no point)
              const int id = f2i(t[j].w);
              r.offer(d, id, kPosPending);
              if (r.id[0] == id) q0 = t[j];
            }
          }
        }
      }
    }
    wave_sync();
  }
  if (pclk) pclk[2] = __builtin_amdgcn_s_memtime();
  // (!Resolve: r.pos stays kPosPending / -1 -- the caller keeps r.id, the
  // original indices, and maps them itself when it needs positions)
  if (Resolve && ok) pix_resolve(bv, pv, r);
  // (the seed lies in the window, so the first is within rc; checked anyway)
  return ok && r.pos[0] >= 0 && margin_sqrt(r.d[0]) * 1.00001f + 1e-30f < rc;
}

// The row mode of the window search (r23): when a wavefront's searching
// lanes are few (<= kRowQ) and every window small (<= kRowPx pixels), each
// query takes a row of 16 lanes -- four at a time -- whose lanes load its
// window's pixels straight from PixView::pts (8 per lane, one memory trip)
// and merge their two nearest by DPP (wave_lex_min<8>): no union box, no
// LDS staging, no per-lane scan of the window.  The same pixels as
// pix_tile_search's window, the same (d2, index) order: the same two
// nearest, the same covered radius rc, the same q0.  handled = false
// (uniform): the wavefront does not qualify, nothing was done.  Measured
// slower (r23c, 172/172 GPU tests bit-identical: k_icp_nn_b 247 -> 266 us,
// 43.5k -> 41.3k it/s; at five waves a SIMD, without its 92 B of spills,
// 261 us): off.
#ifndef RST_PIX_ROWMODE
#define RST_PIX_ROWMODE 0
#endif
constexpr int kRowPx = 16 * 8;
constexpr int kRowQ = 8;
__device__ __forceinline__ float rl_f(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
template <bool Resolve>
__device__ __forceinline__ bool pix_row_search(const BvhView& bv, const PixView& pv, bool act, float qx,
                                               float qy, float qz, float d0, Best2& r, float4& q0, float& rc,
                                               float maxh, bool& handled) {
  const int lane = __lane_id(), row = lane >> 4, sub = lane & 15;
  int a0 = 0, a1 = -1, b0 = 0, b1 = -1;
  float rcl = 0.f;
  const bool ok = act && pix_window(pv, qx, qy, qz, d0, maxh, a0, a1, b0, b1, rcl);
  const int wa = a1 - a0 + 1, cnt = ok ? wa * (b1 - b0 + 1) : 0;
  const uint64_t om = __ballot(ok);
  handled = om != 0 && __popcll(om) <= kRowQ && __ballot(ok && cnt > kRowPx) == 0;
  if (!handled) return false;
  rc = rcl;
  uint64_t rem = om;
  while (rem) {  // (uniform) four queries a round, one a row
    int L[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      L[g] = rem ? (int)__builtin_ctzll(rem) : -1;
      rem &= rem ? rem - 1 : 0;
    }
    // this row's query (its lane's values, read as scalars)
    float rx = 0.f, ry = 0.f, rz = 0.f;
    int ra0 = 0, rb0 = 0, rwa = 1, rcnt = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (L[g] >= 0) {  // (uniform)
        const float x = rl_f(qx, L[g]), y = rl_f(qy, L[g]), z = rl_f(qz, L[g]);
        const int ia = __builtin_amdgcn_readlane(a0, L[g]), ib = __builtin_amdgcn_readlane(b0, L[g]);
        const int iw = __builtin_amdgcn_readlane(wa, L[g]), ic = __builtin_amdgcn_readlane(cnt, L[g]);
        if (row == g) {
          rx = x; ry = y; rz = z;
          ra0 = ia; rb0 = ib; rwa = iw; rcnt = ic;
        }
      }
    }
    Best2 mine;
    mine.init();
    float4 mq = make_float4(NAN, NAN, NAN, 0.f);
    {
      const float rw = 1.0f / (float)max(rwa, 1);
      float4 p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // (every load in flight)
        const int k = sub + 16 * j;
        p[j] = make_float4(NAN, NAN, NAN, 0.f);
        if (k < rcnt) {
          const int rr = (int)(((float)k + 0.5f) * rw);  // k / rwa (exact: k < 2^12)
          p[j] = pv.pts[(int64_t)(rb0 + rr) * pv.w + (ra0 + k - rr * rwa)];
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = d2_ref(rx, ry, rz, p[j].x, p[j].y, p[j].z);
        if (d <= mine.d[1]) {  // (NaN: no point)
          const int id = f2i(p[j].w);
          mine.offer(d, id, kPosPending);
          if (mine.id[0] == id) mq = p[j];
        }
      }
    }
    const int pre = mine.id[0];
    mine = wave_lex_min<8>(mine);
    // the winner's point: the first lane of its row whose own first it was
    const uint64_t hm = __ballot(mine.pos[0] >= 0 && pre == mine.id[0]);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (L[g] >= 0) {  // (uniform)
        const int src = 16 * g;
        const float e0 = rl_f(mine.d[0], src), e1 = rl_f(mine.d[1], src);
        const int i0 = __builtin_amdgcn_readlane(mine.id[0], src), i1 = __builtin_amdgcn_readlane(mine.id[1], src);
        const int p0 = __builtin_amdgcn_readlane(mine.pos[0], src), p1 = __builtin_amdgcn_readlane(mine.pos[1], src);
        const uint64_t rb = (hm >> (16 * g)) & 0xffffull;
        const int w = rb ? 16 * g + (int)__builtin_ctzll(rb) : src;
        const float4 wq = make_float4(rl_f(mq.x, w), rl_f(mq.y, w), rl_f(mq.z, w), rl_f(mq.w, w));
        if (lane == L[g]) {
          r.d[0] = e0;
          r.d[1] = e1;
          r.id[0] = i0;
          r.id[1] = i1;
          r.pos[0] = p0;
          r.pos[1] = p1;
          if (rb) q0 = wq;
        }
      }
    }
  }
  if (Resolve && ok) pix_resolve(bv, pv, r);
  return ok && r.pos[0] >= 0 && margin_sqrt(r.d[0]) * 1.00001f + 1e-30f < rc;
}

// One query per row of 16 lanes (the fallback's short queues): the row's
// lanes split the query's pixel window, then a row-wide (d2, index) merge.
// r holds the seeds (r.d[0] = the seed distance); on true r is the exact two
// nearest within rc.  Whole rows call it (act uniform per row).
__device__ __forceinline__ bool row_pix(const BvhView& bv, const PixView& pv, bool act, float qx,
                                        float qy, float qz, Best2& r, float& rc,
                                        float maxh = RST_PIX_MAX_HALF) {
  const int sub = __lane_id() & 15;
  int a0 = 0, a1 = -1, b0 = 0, b1 = -1;
  rc = 0.f;
  const bool ok = act && pix_window(pv, qx, qy, qz, r.d[0], maxh, a0, a1, b0, b1, rc);
  Best2 mine;
  mine.init();
  const int wa = a1 - a0 + 1;
  const int cnt = ok ? wa * (b1 - b0 + 1) : 0;
  const float rwa = 1.0f / (float)max(wa, 1);
  for (int k0 = 0; k0 < cnt; k0 += 16 * 8) {
    float4 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // 8 pixels per lane in flight
      const int k = k0 + sub + 16 * j;
      p[j] = make_float4(NAN, NAN, NAN, 0.f);
      if (k < cnt) {
        const int rr = (int)(((float)k + 0.5f) * rwa);  // k / wa (exact)
        const int64_t px = (int64_t)(b0 + rr) * pv.w + (a0 + k - rr * wa);
        p[j] = pv.pts[px];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = d2_ref(qx, qy, qz, p[j].x, p[j].y, p[j].z);
      if (d <= mine.d[1]) mine.offer(d, f2i(p[j].w), kPosPending);  // (NaN: no point)
    }
  }
  mine = wave_lex_min<8>(mine);
  if (ok) pix_resolve(bv, pv, mine);
  const bool ex = ok && mine.pos[0] >= 0 && margin_sqrt(mine.d[0]) * 1.00001f + 1e-30f < rc;
  if (ex) r = mine;  // (else r keeps its seeds for the next search)
  return ex;
}

// ---- the ICP loop's candidate lists ----------------------------------------------------
// Exact K nearest of q (r empty: BestK keeps duplicate offers) through the
// leaf adjacency of the leaf holding sorted position `start`: the entries in
// order of box distance, each scanned when its box meets the ball of the
// running K-th distance, until an entry lies beyond that ball (sorted: all
// later ones do too); then the coverage test with the FINAL radius -- every
// point inside the final ball lies in a listed leaf (reach), each listed
// leaf within it was visited with a ball at least as large.  Returns false
// (r only improved) when the ball is not covered.  While the list holds
// fewer than K points the radius is infinite: every entry is scanned.
template <int K>
RST_HD bool adj_knn_search(const BvhView& bv, const AdjView& av, int start, float qx, float qy,
                           float qz, BestK<K>& r) {
  const int nl = bv.nleaves;
  const int L = leaf_of(bv, start);
  const float4 lo = bv.nodes[2 * (nl + L)], hi = bv.nodes[2 * (nl + L) + 1];
  // margins cover float rounding of every distance (rst_bvh.hpp adj_search)
  const float dl = sqrtf(box_d2(qx, qy, qz, lo, hi)) * 1.00001f;
  const float4* e = av.ent + (int64_t)L * kAdjK * 2;
  for (int k0 = 0; k0 < kAdjK; k0 += 4) {
    float4 l[4], h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      l[j] = e[2 * (k0 + j)];
      h[j] = e[2 * (k0 + j) + 1];
    }
    bool stop = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (stop) break;
      const int tag = f2i(h[j].w);
      if (tag < 0 || l[j].w * 0.99999f - dl > r.radius() * 1.00001f + 1e-30f) {
        stop = true;
      } else if (box_d2(qx, qy, qz, l[j], h[j]) <= r.bound()) {
        scan_range_wide(bv, tag >> 5, tag & 31, qx, qy, qz, r);
      }
    }
    if (stop) break;
  }
  return dl + r.radius() * 1.00001f + 1e-30f < av.reach[L] * 0.99999f;
}

// The exact K nearest of one query through the leaf adjacency of the warm
// point's leaf, whole wavefront (the ICP loop's list rebuild): lanes 0..23
// load the 24 entries at once and rank them by box distance to q; leaves
// are then scanned four per load instruction (16 lanes per leaf) in that
// order until the next leaf's box lies beyond the running K-th distance, and
// each batch's points are merged into the list (uniform across the wave) in
// ascending order.  Exact when covered: every point within the final ball
// lies in a listed leaf (reach), and every listed leaf whose box meets the
// final ball was scanned (ascending box order, the ball only shrinks).
// Returns false (L holds what was found) when the ball is not covered.
template <int K>
__device__ __forceinline__ bool nn_wave_knn(const BvhView& bv, const AdjView& av, int warm,
                                            float qx, float qy, float qz, BestK<K>& L,
                                            WnnScratch& ws) {
  const int lane = __lane_id();
  const int nl = bv.nleaves;
  L.init();
  if (bv.m <= 0 || warm < 0 || warm >= bv.m || !finite3(qx, qy, qz)) return false;
  const int H = leaf_of(bv, warm);
  const float4* e = av.ent + (int64_t)H * kAdjK * 2;
  float4 l = make_float4(0.f, 0.f, 0.f, 0.f), h = l;
  int tag = -1;
  if (lane < kAdjK) {
    l = e[2 * lane];
    h = e[2 * lane + 1];
    tag = f2i(h.w);
  }
  const float4 nlo = bv.nodes[2 * (nl + H)], nhi = bv.nodes[2 * (nl + H) + 1];
  const float rch = av.reach[H];
  // margins cover float rounding of every distance (rst_bvh.hpp adj_search)
  const float dl = sqrtf(box_d2(qx, qy, qz, nlo, nhi)) * 1.00001f;
  const bool valid = lane < kAdjK && tag >= 0;
  const float bq = valid ? box_d2(qx, qy, qz, l, h) : FLT_MAX;
  int rank = 0;
#pragma unroll
  for (int j = 0; j < kAdjK; ++j) {
    const float bj = wnn_rl(bq, j);
    rank += ((bj < bq) | ((bj == bq) & (j < lane))) ? 1 : 0;
  }
  const int nv = __popcll(__ballot(valid));
  if (valid) ws.leaf_lo[rank] = make_float4(bq, 0.f, 0.f, i2f(tag));
  wave_sync();
  const int g = lane >> 4, o = lane & 15;
  for (int b0 = 0; b0 < nv; b0 += 4) {
    if (ws.leaf_lo[b0].x > L.bound()) break;  // every later leaf is farther still
    float d = FLT_MAX;
    int id = 0x7fffffff, ps = -1;
    if (b0 + g < nv) {
      const float4 en = ws.leaf_lo[b0 + g];
      const int tg = f2i(en.w);
      if (en.x <= L.bound() && o < (tg & 31)) {
        ps = (tg >> 5) + o;
        const float4 p = bv.pts[ps];
        d = d2_ref(qx, qy, qz, p.x, p.y, p.z);
        id = f2i(p.w);
      }
    }
    // merge the batch: its candidates that beat the K-th, smallest first
    bool live = ps >= 0 && lex_less(d, id, L.d[K - 1], L.id[K - 1]);
    while (__ballot(live)) {
      Best1 c;
      c.d = live ? d : FLT_MAX;
      c.id = live ? id : 0x7fffffff;
      c.pos = live ? ps : -1;
      c = wave_lex_min(c);
      if (!lex_less(c.d, c.id, L.d[K - 1], L.id[K - 1])) break;
      L.offer(c.d, c.id, c.pos);
      live = live && id != c.id && lex_less(d, id, L.d[K - 1], L.id[K - 1]);
    }
  }
  wave_sync();
  return dl + sqrtf(L.bound()) * 1.00001f + 1e-30f < rch * 0.99999f;
}

// The list certificate (icp.hip): a list made at query position c.xyz holds
// every target point with d2 < c.w = R2 (the K-th distance of an exact K-NN
// search; no other point is closer).  For the query now at p, delta =
// |p - c| away, every point off the list is at least sqrt(R2) - delta from
// p; when the list's best point is closer than that by the 1e-5 relative
// margins (float rounding of each distance here is < 1e-6 relative), the
// list's lexicographic minimum is the exact nearest neighbour.
RST_HD bool list_cert_holds(const float4& c, float dbest, float px, float py, float pz) {
  const float ex = px - c.x, ey = py - c.y, ez = pz - c.z;
  const float del = sqrtf((ex * ex + ey * ey) + ez * ez);
  return c.w > 0.0f && sqrtf(dbest) * 1.00001f + del * 1.00001f + 1e-30f < sqrtf(c.w) * 0.99999f;
}

// ---- adjacency build: one wavefront per leaf -------------------------------------
// Range query around box(L) with radius D0 = 3 x its diagonal (halved while
// more than kWnnLeaves leaves fall inside), then the kAdjK nearest of the
// collected leaves by rank.  reach[L] = the (kAdjK+1)-th distance when more
// were collected, else sqrt(D0^2): every leaf not listed is at least that
// far (non-collected leaves have bbd2 > D0^2).  Degenerate cases (empty box,
// persistent overflow) get reach 0: such a leaf never certifies a query.
// Items = the tree nodes [first, 2 first) of one level (first = nleaves:
// the leaves; first = nleaves >> 3: nodes of 8 leaves), L = item index.
__device__ __forceinline__ void leaf_adj_wave(const BvhView& bv, int first, int L,
                                              float4* __restrict__ ent, float* __restrict__ reach,
                                              WnnScratch& ws) {
  const int lane = __lane_id();
  const int nl = first;
  const float4 ql = bv.nodes[2 * (nl + L)], qh = bv.nodes[2 * (nl + L) + 1];
  const float dx = qh.x - ql.x, dy = qh.y - ql.y, dz = qh.z - ql.z;
  const float diag2 = dx * dx + dy * dy + dz * dz;
  float D2 = 9.0f * diag2;  // radius 3 x the item's diagonal, halved on overflow
  int ns = 0;
  bool overflow = !(ql.x <= qh.x) || !(diag2 < FLT_MAX);
  for (int attempt = 0; attempt < 6 && !(!(ql.x <= qh.x) || !(diag2 < FLT_MAX)); ++attempt) {
    const unsigned start = (unsigned)(nl + L);
    const int depth = 31 - __clz(start);
    if (lane < depth) ws.stack[lane] = (int)((start >> (depth - 1 - lane)) ^ 1u);
    if (lane == 0) ws.stack[depth] = (int)start;
    int sp = depth + 1;
    ns = 0;
    overflow = false;
    const uint64_t lt = (1ull << lane) - 1ull;
    wave_sync();
    while (sp > 0 && !overflow) {
      const int k = min(min(kWnnPop, sp), max(1, (kWnnStack - 48 - sp) / 2));
      int node = 0;
      if (lane < k) node = ws.stack[sp - 1 - lane];
      sp -= k;
      wave_sync();
      bool pass = false;
      float b2 = 0.f;
      if (lane < k) {
        b2 = bbd2(ql, qh, bv.nodes[2 * node], bv.nodes[2 * node + 1]);
        pass = b2 <= D2;
      }
      const bool isleaf = node >= nl;
      const uint64_t im = __ballot(pass && !isleaf);
      const uint64_t lm = __ballot(pass && isleaf);
      if (ns + __popcll(lm) > kWnnLeaves) {
        overflow = true;
        break;
      }
      if (pass && !isleaf) {
        const int rk = __popcll(im & lt);
        ws.stack[sp + 2 * rk] = 2 * node + 1;
        ws.stack[sp + 2 * rk + 1] = 2 * node;
      }
      if (pass && isleaf) ws.leaf_lo[ns + __popcll(lm & lt)] = make_float4(b2, 0.f, 0.f, i2f(node - nl));
      sp += 2 * __popcll(im);
      ns += __popcll(lm);
      wave_sync();
    }
    if (!overflow) break;
    D2 *= 0.25f;
  }
  float4* e = ent + (int64_t)L * kAdjK * 2;
  if (overflow) {
    if (lane < kAdjK) {
      e[2 * lane] = make_float4(0.f, 0.f, 0.f, INFINITY);
      e[2 * lane + 1] = make_float4(0.f, 0.f, 0.f, i2f(-1));
    }
    if (lane == 0) reach[L] = 0.0f;
    return;
  }
  wave_sync();
  // rank of each collected leaf in (bbd2, index) order
  float rk_b2 = -1.f;  // bbd2 of the element ranked kAdjK (the reach)
  for (int s = lane; s < kWnnLeaves; s += 64) {
    int rank = 1 << 30;
    float mb = 0.f;
    int mid = 0;
    if (s < ns) {
      const float4 me = ws.leaf_lo[s];
      mb = me.x;
      mid = f2i(me.w);
      rank = 0;
      for (int t = 0; t < ns; ++t) {
        const float4 o = ws.leaf_lo[t];
        rank += lex_less(o.x, f2i(o.w), mb, mid) ? 1 : 0;
      }
    }
    if (rank < kAdjK) {
      e[2 * rank] = make_float4(bv.nodes[2 * (nl + mid)].x, bv.nodes[2 * (nl + mid)].y,
                                bv.nodes[2 * (nl + mid)].z, sqrtf(mb));
      const float4 h = bv.nodes[2 * (nl + mid) + 1];
      const int tag = first == bv.nleaves ? leaf_tag(bv, mid) : mid;
      e[2 * rank + 1] = make_float4(h.x, h.y, h.z, i2f(tag));
    }
    if (rank == kAdjK) rk_b2 = mb;
  }
  if (lane >= ns && lane < kAdjK) {
    e[2 * lane] = make_float4(0.f, 0.f, 0.f, INFINITY);
    e[2 * lane + 1] = make_float4(0.f, 0.f, 0.f, i2f(-1));
  }
  const float kth = wnn_max_f(rk_b2);
  if (lane == 0) reach[L] = ns > kAdjK ? sqrtf(kth) : sqrtf(D2);
}

}  // namespace rst
