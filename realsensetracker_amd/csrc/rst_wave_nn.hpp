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
//   2. region = AABB of all lanes' balls (radius sqrt(bound), inflated);
//   3. staging walk: LIFO stack of node ids in LDS, popped up to 32 at a
//      time -- lane t loads node t's box (one coalesced load per round, all
//      in flight together), keeps it if it meets the region; internal nodes
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
// Exactness: a node is dropped only if its box misses the region, i.e. for
// every lane its box_d2 exceeds that lane's bound; a staged leaf is skipped
// only if no lane's box_d2 <= bound.  Bounds only decrease, so every point
// not offered is strictly worse than the final answer (same argument as the
// tree walks of rst_bvh.hpp, which tests/cpp/bvh_selftest.cpp checks).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>

#include "rst_bvh.hpp"

namespace rst {

constexpr int kWnnStack = 512;   // node ids per wave (see the overflow rule)
constexpr int kWnnLeaves = 64;   // staged leaves per flush
constexpr int kWnnPop = 32;      // nodes tested per staging round

struct WnnScratch {              // per-wave LDS (4 KB)
  int stack[kWnnStack];
  float4 leaf_lo[kWnnLeaves];    // .w = leaf index bits
  float4 leaf_hi[kWnnLeaves];    // .w = point count bits
};

__device__ __forceinline__ float wnn_rl(float v, int l) {
  return i2f(__builtin_amdgcn_readlane(f2i(v), l));
}
__device__ __forceinline__ int wnn_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wnn_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wnn_min_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wnn_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

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

__device__ __forceinline__ WnnRegion wnn_region(bool act, float qx, float qy, float qz,
                                                float bound) {
  // inflate so float rounding can never drop a node some lane needs
  const float rad = act ? sqrtf(bound) * 1.0001f + 1e-20f : 0.0f;
  WnnRegion g;
  g.lx = wnn_min_f(act ? qx - rad : FLT_MAX);
  g.ly = wnn_min_f(act ? qy - rad : FLT_MAX);
  g.lz = wnn_min_f(act ? qz - rad : FLT_MAX);
  g.hx = wnn_max_f(act ? qx + rad : -FLT_MAX);
  g.hy = wnn_max_f(act ? qy + rad : -FLT_MAX);
  g.hz = wnn_max_f(act ? qz + rad : -FLT_MAX);
  return g;
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
// staging rounds, nodes tested, leaves staged, leaves scanned, flushes,
// active lanes, lanes with no finite bound, region extent (um, max axis).
__device__ __forceinline__ void nn_wave_region(const BvhView& bv, bool act, float qx, float qy,
                                            float qz, Best1& r, WnnScratch& ws,
                                            int* stats = nullptr) {
  const int lane = __lane_id();
  const int nl = bv.nleaves;
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
  __builtin_amdgcn_wave_barrier();
  WnnRegion reg = wnn_region(act, qx, qy, qz, r.d);
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
      const int k = sp > kWnnStack - 64 ? 1 : min(kWnnPop, sp);
      ++st_rounds;
      st_nodes += k;
      int node = 0;
      if (lane < k) node = ws.stack[sp - 1 - lane];
      sp -= k;
      __builtin_amdgcn_wave_barrier();
      bool pass = false;
      float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
      if (lane < k) {
        lo = bv.nodes[2 * node];
        hi = bv.nodes[2 * node + 1];
        pass = reg.meets(lo, hi);
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
      __builtin_amdgcn_wave_barrier();
    }
    if (ns > kWnnLeaves - kWnnPop || (sp == 0 && ns > 0)) {
      st_scanned += wnn_flush(bv, ws, ns, act, qx, qy, qz, r);
      ++st_flush;
      ns = 0;
      reg = wnn_region(act, qx, qy, qz, r.d);
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (stats && lane == 0) {
    stats[0] = st_rounds;
    stats[1] = st_nodes;
    stats[2] = st_staged;
    stats[3] = st_scanned;
    stats[4] = st_flush;
  }
}

}  // namespace rst
