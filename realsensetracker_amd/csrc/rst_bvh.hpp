// rst_bvh.hpp -- the exact-NN index over a target cloud and its searches.
//
// Replaces the reference's nanoflann kd-tree (KDTree3f{dst,16},
// kdtree.hpp:27-57; query at align_icp.cpp:112).  The index is an implicit
// heap BVH over the Morton-sorted target points:
//   root = node 1, children 2k / 2k+1, leaves = nodes [nl, 2nl), nl = 2^lg;
//   node k = two float4: lo (x, y, z, split) and hi (x, y, z, axis bits);
//   leaf L holds sorted points [L*m >> lg, (L+1)*m >> lg)  (8..16 points).
//
// Every search here is EXACT: the result is the lexicographic minimum of
// (d2, original index) over all points with d2 < FLT_MAX, where d2 is
// nanoflann's float ((dx*dx + dy*dy) + dz*dz).  Searches differ only in the
// order they visit subtrees, which changes the work, never the answer:
//   descend(root)      top-down stackless walk of one subtree (near child
//                      first, parent recovered as k >> 1);
//   search_from(pos)   bottom-up from the leaf holding sorted position pos
//                      (a warm candidate: last ICP iteration's neighbour,
//                      or the query point itself for kNN normals): that
//                      leaf, then the sibling subtree of every ancestor.
//                      With a good warm candidate the bound is tight from
//                      the start and only the few low siblings that touch
//                      the query ball are entered -- a short dependent-load
//                      chain per lane instead of a root-to-leaf walk.
// Written __host__ __device__ so tests/cpp/bvh_selftest.cpp checks the same
// code against brute force on the CPU.
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#define RST_HD __host__ __device__ __forceinline__

namespace rst {

constexpr int kLeafTarget = 16;  // nanoflann leaf_max_size at align_icp.cpp:165

RST_HD int f2i(float f) { return __builtin_bit_cast(int, f); }
RST_HD float i2f(int i) { return __builtin_bit_cast(float, i); }
RST_HD bool finite3(float x, float y, float z) {
  return __builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z);
}

// nanoflann L2_Adaptor::evalMetric for DIM=3: ((dx*dx + dy*dy) + dz*dz),
// d = query - point (kdtree.hpp:51-57).  The library is compiled with
// -ffp-contract=off, so every operation rounds as written.
RST_HD float d2_ref(float qx, float qy, float qz, float px, float py, float pz) {
  const float dx = qx - px;
  const float dy = qy - py;
  const float dz = qz - pz;
  float r = dx * dx;
  r = r + dy * dy;
  r = r + dz * dz;
  return r;
}

// Lower bound of d2_ref over every point of an AABB: per-axis gaps are
// monotone in float, so this never exceeds any contained point's d2_ref.
RST_HD float box_d2(float qx, float qy, float qz, const float4& lo, const float4& hi) {
  const float ex = fmaxf(fmaxf(lo.x - qx, qx - hi.x), 0.0f);
  const float ey = fmaxf(fmaxf(lo.y - qy, qy - hi.y), 0.0f);
  const float ez = fmaxf(fmaxf(lo.z - qz, qz - hi.z), 0.0f);
  float r = ex * ex;
  r = r + ey * ey;
  r = r + ez * ez;
  return r;
}

struct BvhView {
  const float4* __restrict__ pts;    // [m] sorted points, .w = original index bits
  const float4* __restrict__ nodes;  // [2 * 2nl]
  int32_t m;
  int32_t nleaves;
  int32_t lg;                        // nleaves = 1 << lg
  int32_t pad;
};

RST_HD int leaf_begin(const BvhView& bv, int L) { return (int)(((int64_t)L * bv.m) >> bv.lg); }

// Leaf holding sorted position p: the largest L with leaf_begin(L) <= p.
RST_HD int leaf_of(const BvhView& bv, int p) {
  int L = (int)((((double)p + 1.0) * (double)bv.nleaves - 1.0) / (double)bv.m);
  L = L < 0 ? 0 : (L >= bv.nleaves ? bv.nleaves - 1 : L);
  while (L > 0 && leaf_begin(bv, L) > p) --L;
  while (L + 1 < bv.nleaves && leaf_begin(bv, L + 1) <= p) ++L;
  return L;
}

RST_HD int near_child(int k, const float4& lo, const float4& hi, float qx, float qy, float qz) {
  const int ab = f2i(hi.w);
  const int ax = ab & 3;
  const float qa = ax == 0 ? qx : (ax == 1 ? qy : qz);
  const bool q_low = qa < lo.w;
  const bool left_low = (ab & 4) == 0;
  return (q_low == left_low) ? (2 * k) : (2 * k + 1);
}

// ---- result sets ---------------------------------------------------------------
// Lexicographic (d2, id) order; only d2 < FLT_MAX is ever admitted (what
// nanoflann's KNNResultSet does with its FLT_MAX-initialised slots).
RST_HD bool lex_less(float a, int ia, float b, int ib) {
  return (a < b) || ((a == b) && (ia < ib));
}

struct Best1 {
  float d;
  int id;
  int pos;
  RST_HD void init() {
    d = FLT_MAX;
    id = 0;
    pos = -1;
  }
  RST_HD float bound() const { return d; }
  RST_HD void offer(float d2, int id_, int pos_) {
    const bool b = lex_less(d2, id_, d, id);
    d = b ? d2 : d;
    id = b ? id_ : id;
    pos = b ? pos_ : pos;
  }
};

// K best, sorted; branch-free insertion with static indices (registers).
template <int K>
struct BestK {
  float d[K];
  int id[K];
  int pos[K];
  RST_HD void init() {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      d[j] = FLT_MAX;
      id[j] = 0x7fffffff;
      pos[j] = -1;
    }
  }
  RST_HD float bound() const { return d[K - 1]; }
  RST_HD void offer(float nd, int nid, int np) {
    if (!(nd < FLT_MAX) || !lex_less(nd, nid, d[K - 1], id[K - 1])) return;
#pragma unroll
    for (int j = K - 1; j >= 1; --j) {
      const bool shift = lex_less(nd, nid, d[j - 1], id[j - 1]);
      const bool here = !shift && lex_less(nd, nid, d[j], id[j]);
      d[j] = shift ? d[j - 1] : (here ? nd : d[j]);
      id[j] = shift ? id[j - 1] : (here ? nid : id[j]);
      pos[j] = shift ? pos[j - 1] : (here ? np : pos[j]);
    }
    if (lex_less(nd, nid, d[0], id[0])) {
      d[0] = nd;
      id[0] = nid;
      pos[0] = np;
    }
  }
};

// ---- traversal ---------------------------------------------------------------------
template <class R>
RST_HD void scan_leaf(const BvhView& bv, int L, float qx, float qy, float qz, R& res) {
  const int b = leaf_begin(bv, L);
  const int e = leaf_begin(bv, L + 1);
  for (int i = b; i < e; ++i) {
    const float4 p = bv.pts[i];
    res.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), i);
  }
}

// Stackless walk of the subtree rooted at `root` (entered from its parent):
// near child first; a node is skipped when its box bound exceeds the
// current result bound (strictly: an equal-d2 point may still win on index).
template <class R>
RST_HD void descend(const BvhView& bv, int root, float qx, float qy, float qz, R& res) {
  const int nl = bv.nleaves;
  const int top = root >> 1;
  int cur = root, prev = top;
  do {
    const int parent = cur >> 1;
    const float4 lo = bv.nodes[2 * cur];
    const float4 hi = bv.nodes[2 * cur + 1];
    int next;
    if (prev == parent) {
      if (box_d2(qx, qy, qz, lo, hi) > res.bound()) {
        next = parent;
      } else if (cur >= nl) {
        scan_leaf(bv, cur - nl, qx, qy, qz, res);
        next = parent;
      } else {
        next = near_child(cur, lo, hi, qx, qy, qz);
      }
    } else {
      const int nc = near_child(cur, lo, hi, qx, qy, qz);
      next = (prev == nc) ? (prev ^ 1) : parent;
    }
    prev = cur;
    cur = next;
  } while (cur != top);
}

// Bottom-up exact search from the leaf of sorted position `start` (valid,
// 0 <= start < m): the start leaf, then each ancestor's other child.  The
// start leaf plus those siblings partition the tree, so nothing is missed.
template <class R>
RST_HD void search_from(const BvhView& bv, int start, float qx, float qy, float qz, R& res) {
  const int nl = bv.nleaves;
  int node = nl + leaf_of(bv, start);
  scan_leaf(bv, node - nl, qx, qy, qz, res);
  while (node > 1) {
    descend(bv, node ^ 1, qx, qy, qz, res);
    node >>= 1;
  }
}

// Exact search of the whole index: bottom-up from `warm` when given (>= 0),
// else top-down from the root.  Non-finite queries find nothing.
template <class R>
RST_HD void search(const BvhView& bv, int warm, float qx, float qy, float qz, R& res) {
  if (bv.m <= 0 || !finite3(qx, qy, qz)) return;
  if (warm >= 0 && warm < bv.m)
    search_from(bv, warm, qx, qy, qz, res);
  else
    descend(bv, 1, qx, qy, qz, res);
}

// ---- build: internal node from its two children ------------------------------------
// lo/hi = union box; split = midpoint of the children's centres along the
// axis of largest centre separation; axis bits: 0-1 axis, bit 2 set when the
// left child lies on the high side.  Empty children (lo.x > hi.x) steer the
// walk to the non-empty one.
RST_HD void make_internal(float4* nodes, int k) {
  const float4 l0 = nodes[2 * (2 * k)], h0 = nodes[2 * (2 * k) + 1];
  const float4 l1 = nodes[2 * (2 * k + 1)], h1 = nodes[2 * (2 * k + 1) + 1];
  float4 lo, hi;
  lo.x = fminf(l0.x, l1.x); lo.y = fminf(l0.y, l1.y); lo.z = fminf(l0.z, l1.z);
  hi.x = fmaxf(h0.x, h1.x); hi.y = fmaxf(h0.y, h1.y); hi.z = fmaxf(h0.z, h1.z);
  const bool e0 = !(l0.x <= h0.x), e1 = !(l1.x <= h1.x);
  float split;
  int ab;
  if (e0 || e1) {
    ab = 0;
    split = e1 ? INFINITY : -INFINITY;
  } else {
    const float c0[3] = {0.5f * (l0.x + h0.x), 0.5f * (l0.y + h0.y), 0.5f * (l0.z + h0.z)};
    const float c1[3] = {0.5f * (l1.x + h1.x), 0.5f * (l1.y + h1.y), 0.5f * (l1.z + h1.z)};
    int ax = 0;
    float best = fabsf(c1[0] - c0[0]);
    for (int a = 1; a < 3; ++a)
      if (fabsf(c1[a] - c0[a]) > best) {
        best = fabsf(c1[a] - c0[a]);
        ax = a;
      }
    split = 0.5f * (c0[ax] + c1[ax]);
    ab = ax | (c0[ax] <= c1[ax] ? 0 : 4);
  }
  lo.w = split;
  hi.w = i2f(ab);
  nodes[2 * k] = lo;
  nodes[2 * k + 1] = hi;
}

// Leaf box over finite points only (non-finite points sort last and are
// never admitted by d2 < FLT_MAX anyway).
RST_HD void make_leaf(const BvhView& bv, float4* nodes, int L) {
  float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.0f);
  float4 hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
  const int b = leaf_begin(bv, L), e = leaf_begin(bv, L + 1);
  for (int i = b; i < e; ++i) {
    const float4 p = bv.pts[i];
    if (!finite3(p.x, p.y, p.z)) continue;
    lo.x = fminf(lo.x, p.x); lo.y = fminf(lo.y, p.y); lo.z = fminf(lo.z, p.z);
    hi.x = fmaxf(hi.x, p.x); hi.y = fmaxf(hi.y, p.y); hi.z = fmaxf(hi.z, p.z);
  }
  const int k = bv.nleaves + L;
  nodes[2 * k] = lo;
  nodes[2 * k + 1] = hi;
}

}  // namespace rst
