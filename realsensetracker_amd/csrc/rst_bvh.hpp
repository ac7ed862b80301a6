// rst_bvh.hpp -- the exact-NN index over a target cloud and its searches.
//
// Replaces the reference's nanoflann kd-tree (KDTree3f{dst,16},
// kdtree.hpp:27-57; query at align_icp.cpp:112).  The index is an implicit
// heap BVH over the Morton-sorted target points:
//   root = node 1, children 2k / 2k+1, leaves = nodes [nl, 2nl), nl = 2^lg;
//   node k = two float4: lo (x, y, z, split) and hi (x, y, z, axis bits);
//   leaf L holds sorted points [lstart[L], lstart[L+1]) (1..16 points;
//   leaves past the last are empty).  Leaves are compact: the Morton order
//   is cut wherever it leaves a 4x4x4-cell block of the code grid (the
//   Z-curve jumps across space there on a 2.5D surface) and every run is
//   chopped into <= 16-point pieces -- see leaf_cut().
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

// Sorted point arrays carry kPtsPad float4 of padding past m, so a leaf scan
// may load a full batch from one base address without clamping indices.
constexpr int kPtsPad = 16;

struct BvhView {
  const float4* __restrict__ pts;    // [m] sorted points, .w = original index bits
  const float4* __restrict__ nodes;  // [2 * 2nl]
  const uint32_t* __restrict__ codes;  // [m] sorted Morton codes (may be null)
  const int32_t* __restrict__ lstart;  // [nl + 1] first point of each leaf
  const int32_t* __restrict__ pleaf;   // [m] leaf of each sorted point
  const float* __restrict__ bbox;    // [6] the codes' quantisation box (may be null)
  int32_t m;
  int32_t nleaves;
  int32_t lg;                        // nleaves = 1 << lg
  int32_t pad;
};

// A target prepared from a depth frame keeps its pixel grid: map[p] = the
// sorted position of grid pixel p's point (-1: no valid depth), p = vl * w +
// ul on the level grid (pixel (s ul, s vl) of the full image, intrinsics of
// the full image).  Projecting a query through it gives a candidate near its
// nearest neighbour (a warm start), and the grid's pixel windows answer exact
// searches (pix_tile_search, rst_wave_nn.hpp).  pts[p] = the point of pixel p
// (its sorted point, .w = original index bits; NaN where map[p] = -1), so a
// window is staged with one load per pixel and map, in parallel.
struct PixView {
  const int32_t* __restrict__ map;  // null: the target has no pixel grid
  const float4* __restrict__ pts;   // [w h] grid pixel p's point (x, y, z, original index bits)
  const int32_t* __restrict__ inv;  // [m] original index -> sorted position (the target's)
  float fx, fy, cx, cy;
  int32_t w, h, s;
  int32_t pad;
};

// ---- Morton order ------------------------------------------------------------------
RST_HD uint32_t spread10(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// 30-bit code of a point quantised to 1024^3 cells over the cube of side
// max extent at bbox lo; non-finite points sort last.
RST_HD uint32_t morton_code(float x, float y, float z, const float* bbox) {
  const float lx = bbox[0], ly = bbox[1], lz = bbox[2];
  const float ext = fmaxf(fmaxf(bbox[3] - lx, bbox[4] - ly), bbox[5] - lz);
  const float sc = ext > 0.0f ? 1023.0f / ext : 0.0f;
  if (!finite3(x, y, z)) return 0x3fffffffu;
  const uint32_t qx = (uint32_t)fminf(fmaxf((x - lx) * sc, 0.0f), 1023.0f);
  const uint32_t qy = (uint32_t)fminf(fmaxf((y - ly) * sc, 0.0f), 1023.0f);
  const uint32_t qz = (uint32_t)fminf(fmaxf((z - lz) * sc, 0.0f), 1023.0f);
  return (spread10(qx) << 2) | (spread10(qy) << 1) | spread10(qz);
}

// Cold start: the sorted position whose Morton code is nearest to the
// query's (lower bound, clamped) -- usually a point of the same small cell,
// a cheap first bound for the exact searches.
RST_HD int morton_seed(const BvhView& bv, float qx, float qy, float qz) {
  const uint32_t c = morton_code(qx, qy, qz, bv.bbox);
  int lo = 0, hi = bv.m;  // first code >= c in [lo, hi]
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (bv.codes[mid] < c)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < bv.m ? lo : bv.m - 1;
}

RST_HD int leaf_begin(const BvhView& bv, int L) { return bv.lstart[L]; }
RST_HD int leaf_of(const BvhView& bv, int p) { return bv.pleaf[p]; }

// Leaf layout rule: a leaf starts at sorted position i when i begins a new
// block of the code grid (code >> kLeafCellShift differs from i-1's) or
// when kLeafTarget points of the current block have been taken.
// seg = first position of i's block.
constexpr int kLeafCellShift = 9;
RST_HD bool leaf_cut(const uint32_t* codes, int i, int seg) {
  return i == 0 || (codes[i] >> kLeafCellShift) != (codes[i - 1] >> kLeafCellShift) ||
         ((i - seg) % kLeafTarget) == 0;
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
  return (a < b) | ((a == b) & (ia < ib));  // bitwise: no branches on the GPU
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
  RST_HD float radius() const { return sqrtf(d); }
  RST_HD void offer(float d2, int id_, int pos_) {
    const bool b = lex_less(d2, id_, d, id);
    d = b ? d2 : d;
    id = b ? id_ : id;
    pos = b ? pos_ : pos;
  }
};

// The two best (d2, id), sorted.  Offering a point already held (same id)
// changes nothing, so every lane of a wave may start from the same entries
// and a wave merge (wave_lex_min) may see a point twice.  bound() is the
// second distance: a search pruned with it finds both exactly.
struct Best2 {
  float d[2];
  int id[2];
  int pos[2];
  RST_HD void init() {
    d[0] = d[1] = FLT_MAX;
    id[0] = id[1] = 0x7fffffff;
    pos[0] = pos[1] = -1;
  }
  RST_HD float bound() const { return d[1]; }
  RST_HD float radius() const { return sqrtf(d[1]); }
  RST_HD void offer(float nd, int nid, int np) {
    // (nid == id[1] is never lex_less than itself)
    const bool b1 = (nid != id[0]) && lex_less(nd, nid, d[1], id[1]);
    const bool b0 = b1 && lex_less(nd, nid, d[0], id[0]);
    d[1] = b0 ? d[0] : (b1 ? nd : d[1]);
    id[1] = b0 ? id[0] : (b1 ? nid : id[1]);
    pos[1] = b0 ? pos[0] : (b1 ? np : pos[1]);
    d[0] = b0 ? nd : d[0];
    id[0] = b0 ? nid : id[0];
    pos[0] = b0 ? np : pos[0];
  }
  RST_HD Best1 first() const {
    Best1 b;
    b.d = d[0];
    b.id = pos[0] >= 0 ? id[0] : 0;
    b.pos = pos[0];
    return b;
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
  RST_HD float radius() const { return sqrtf(d[K - 1]); }
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

// search_from with every ancestor's sibling box loaded up front (the loads
// are independent, so one latency instead of one per level); only the
// siblings whose box is within the bound -- usually a few low ones -- are
// then walked.  Same result as search_from.
constexpr int kMaxDepth = 28;
template <class R>
RST_HD void search_from_fast(const BvhView& bv, int start, float qx, float qy, float qz, R& res) {
  const int nl = bv.nleaves;
  const int leafnode = nl + leaf_of(bv, start);
  scan_leaf(bv, leafnode - nl, qx, qy, qz, res);
  const int depth = 31 - __builtin_clz((unsigned)leafnode);
  float sb[kMaxDepth];
#pragma unroll
  for (int k = 0; k < kMaxDepth; ++k) {
    sb[k] = FLT_MAX;
    if (k < depth) {
      const int sib = (leafnode >> k) ^ 1;
      sb[k] = box_d2(qx, qy, qz, bv.nodes[2 * sib], bv.nodes[2 * sib + 1]);
    }
  }
#pragma unroll
  for (int k = 0; k < kMaxDepth; ++k)
    if (k < depth && sb[k] <= res.bound()) descend(bv, (leafnode >> k) ^ 1, qx, qy, qz, res);
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

// ---- leaf adjacency: the tracking index ----------------------------------------------
// ICP queries move little between iterations, so a lane's last neighbour is
// a good start and the exact answer lies in a small ball around the query.
// For every leaf L the build stores up to kAdjK nearby leaves by box-to-box
// distance (ascending, L itself first), each entry carrying that leaf's
// box, and reach[L] such that every leaf NOT listed has bbd >= reach[L].  A
// query whose ball (radius sqrt(bound)) satisfies
//     dist(q, box(L)) + sqrt(bound) < reach[L]
// is then answered exactly by the listed leaves alone (any point within
// the ball lies in a leaf whose box is closer to box(L) than reach[L]), and
// the scan stops at the first entry with bbd - dist(q, box(L)) > sqrt(bound)
// (entries are sorted, so no later box can touch the ball either).
constexpr int kAdjK = 24;

// The same index one level up (items = nodes of 2^kAdj2Shift leaves) gives
// the far queries (frame borders, occlusions, early iterations) a reach
// several times larger.
// Level 3 (items = nodes of 2^kAdj3Shift leaves) covers what is left:
// first iterations from a poor pose and the farthest outliers.
constexpr int kAdj2Shift = 3;
constexpr int kAdj3Shift = 6;

struct AdjView {
  // [nl * kAdjK * 2]: entry = (lo.xyz, bbd) (hi.xyz, leaf index bits); leaf -1 = none
  const float4* __restrict__ ent;
  const float* __restrict__ reach;   // [nl]
  const float4* __restrict__ ent2;   // [(nl >> kAdj2Shift) * kAdjK * 2]
  const float* __restrict__ reach2;  // [nl >> kAdj2Shift] (0 when nl is too small)
  const float4* __restrict__ ent3;   // [(nl >> kAdj3Shift) * kAdjK * 2]
  const float* __restrict__ reach3;  // [nl >> kAdj3Shift] (0 when nl is too small)
};

// Box-to-box distance squared (0 when they overlap; +inf when either box
// is empty, i.e. lo > hi).
RST_HD float bbd2(const float4& l1, const float4& h1, const float4& l2, const float4& h2) {
  const float ex = fmaxf(fmaxf(l2.x - h1.x, l1.x - h2.x), 0.0f);
  const float ey = fmaxf(fmaxf(l2.y - h1.y, l1.y - h2.y), 0.0f);
  const float ez = fmaxf(fmaxf(l2.z - h1.z, l1.z - h2.z), 0.0f);
  float r = ex * ex;
  r = r + ey * ey;
  r = r + ez * ez;
  return r;
}

// Entry tag (hi.w bits): at the leaf level the listed leaf's point range,
// begin * 32 + count (count <= 16; begin < 2^26), so a scan needs no further
// lookup; at levels 2/3 the item index.  -1 = no entry.
RST_HD int leaf_tag(const BvhView& bv, int X) {
  const int b = leaf_begin(bv, X);
  return b * 32 + (leaf_begin(bv, X + 1) - b);
}

RST_HD void adj_put(float4* ent, int L, int k, int tag, float bbd, const float4& lo,
                    const float4& hi) {
  float4* e = ent + ((int64_t)L * kAdjK + k) * 2;
  e[0] = make_float4(lo.x, lo.y, lo.z, bbd);
  e[1] = make_float4(hi.x, hi.y, hi.z, i2f(tag));
}

// Offer the sorted points [b, b + n) (one leaf).
template <class R>
RST_HD void scan_range(const BvhView& bv, int b, int n, float qx, float qy, float qz, R& res) {
  for (int i = b; i < b + n; ++i) {
    const float4 p = bv.pts[i];
    res.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), i);
  }
}

// The K nearest leaves of leaf L by bbd2 (items = leaves, id = leaf index):
// bottom-up from L like search_from, pruning subtrees by bbd2 to their box.
// (Reference builder for tests; the GPU builds with rst_wave_nn.hpp.)
template <class R>
RST_HD void leaf_descend(const BvhView& bv, int first, int root, const float4& ql, const float4& qh,
                         R& res) {
  const int nl = first;
  const int top = root >> 1;
  const float cx = 0.5f * (ql.x + qh.x), cy = 0.5f * (ql.y + qh.y), cz = 0.5f * (ql.z + qh.z);
  int cur = root, prev = top;
  do {
    const int parent = cur >> 1;
    const float4 lo = bv.nodes[2 * cur];
    const float4 hi = bv.nodes[2 * cur + 1];
    int next;
    if (prev == parent) {
      const float b = bbd2(ql, qh, lo, hi);
      if (b > res.bound()) {
        next = parent;
      } else if (cur >= nl) {
        res.offer(b, cur - nl, cur - nl);
        next = parent;
      } else {
        next = near_child(cur, lo, hi, cx, cy, cz);
      }
    } else {
      const int nc = near_child(cur, lo, hi, cx, cy, cz);
      next = (prev == nc) ? (prev ^ 1) : parent;
    }
    prev = cur;
    cur = next;
  } while (cur != top);
}

// items = nodes [first, 2 first) (first = nleaves: the leaves)
template <class R>
RST_HD void leaf_knn(const BvhView& bv, int first, int L, R& res) {
  int node = first + L;
  const float4 ql = bv.nodes[2 * node], qh = bv.nodes[2 * node + 1];
  res.offer(bbd2(ql, qh, ql, qh), L, L);
  while (node > 1) {
    leaf_descend(bv, first, node ^ 1, ql, qh, res);
    node >>= 1;
  }
}

// Adjacency record of leaf L from its K+1 nearest (sorted) leaves.
template <int K1>
RST_HD void adj_store(const BvhView& bv, int first, const BestK<K1>& r, int L, float4* ent,
                      float* reach) {
  static_assert(K1 == kAdjK + 1, "list length");
  const int nl = first;
  for (int j = 0; j < kAdjK; ++j) {
    const int X = r.pos[j] >= 0 ? r.id[j] : -1;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const int tag = X < 0 ? -1 : (first == bv.nleaves ? leaf_tag(bv, X) : X);
    adj_put(ent, L, j, tag, X >= 0 ? sqrtf(r.d[j]) : INFINITY, X >= 0 ? bv.nodes[2 * (nl + X)] : z,
            X >= 0 ? bv.nodes[2 * (nl + X) + 1] : z);
  }
  reach[L] = r.pos[kAdjK] >= 0 ? sqrtf(r.d[kAdjK]) : INFINITY;
}

// Exact search through the adjacency of the leaf holding sorted position
// `start` (res already holds at least that point's offer, or a smaller
// bound).  Returns false, having offered nothing, when the query ball is
// not covered -- the caller then needs a full search.
template <class R>
RST_HD bool adj_search(const BvhView& bv, const AdjView& av, int start, float qx, float qy,
                       float qz, R& res) {
  const int nl = bv.nleaves;
  const int L = leaf_of(bv, start);
  const float4 lo = bv.nodes[2 * (nl + L)], hi = bv.nodes[2 * (nl + L) + 1];
  // margins cover float rounding of every distance below (relative 1e-5)
  const float dl = sqrtf(box_d2(qx, qy, qz, lo, hi)) * 1.00001f;
  const float rb = sqrtf(res.bound()) * 1.00001f + 1e-30f;
  if (!(dl + rb < av.reach[L] * 0.99999f)) return false;
  const float4* e = av.ent + (int64_t)L * kAdjK * 2;
  for (int k = 0; k < kAdjK; ++k) {
    const float4 l = e[2 * k], h = e[2 * k + 1];
    const int tag = f2i(h.w);
    if (tag < 0) break;
    if (l.w * 0.99999f - dl > sqrtf(res.bound()) * 1.00001f + 1e-30f) break;
    if (box_d2(qx, qy, qz, l, h) <= res.bound()) scan_range(bv, tag >> 5, tag & 31, qx, qy, qz, res);
  }
  return true;
}

// The same through the level-2 index: entries are nodes of 2^kAdj2Shift
// leaves; a listed node touching the ball has each of its leaves box-tested
// and scanned.  Level-2 nodes partition the leaves, so the coverage argument
// is unchanged.
template <class R>
RST_HD bool adj2_search(const BvhView& bv, const AdjView& av, int start, float qx, float qy,
                        float qz, R& res) {
  const int nl = bv.nleaves;
  if (nl < (1 << kAdj2Shift)) return false;
  const int first = nl >> kAdj2Shift;
  const int N = (nl + leaf_of(bv, start)) >> kAdj2Shift;
  const float4 lo = bv.nodes[2 * N], hi = bv.nodes[2 * N + 1];
  const float dl = sqrtf(box_d2(qx, qy, qz, lo, hi)) * 1.00001f;
  const float rb = sqrtf(res.bound()) * 1.00001f + 1e-30f;
  if (!(dl + rb < av.reach2[N - first] * 0.99999f)) return false;
  const float4* e = av.ent2 + (int64_t)(N - first) * kAdjK * 2;
  for (int k = 0; k < kAdjK; ++k) {
    const float4 l = e[2 * k], h = e[2 * k + 1];
    const int X = f2i(h.w);
    if (X < 0) break;
    if (l.w * 0.99999f - dl > sqrtf(res.bound()) * 1.00001f + 1e-30f) break;
    if (!(box_d2(qx, qy, qz, l, h) <= res.bound())) continue;
    const int leaf0 = ((first + X) << kAdj2Shift) - nl;
    for (int j = 0; j < (1 << kAdj2Shift); ++j) {
      const int Lj = leaf0 + j;
      if (box_d2(qx, qy, qz, bv.nodes[2 * (nl + Lj)], bv.nodes[2 * (nl + Lj) + 1]) <= res.bound())
        scan_leaf(bv, Lj, qx, qy, qz, res);
    }
  }
  return true;
}

// Level 3: listed nodes touching the ball are walked exactly (descend).
template <class R>
RST_HD bool adj3_search(const BvhView& bv, const AdjView& av, int start, float qx, float qy,
                        float qz, R& res) {
  const int nl = bv.nleaves;
  if (nl < (1 << kAdj3Shift)) return false;
  const int first = nl >> kAdj3Shift;
  const int N = (nl + leaf_of(bv, start)) >> kAdj3Shift;
  const float4 lo = bv.nodes[2 * N], hi = bv.nodes[2 * N + 1];
  const float dl = sqrtf(box_d2(qx, qy, qz, lo, hi)) * 1.00001f;
  const float rb = sqrtf(res.bound()) * 1.00001f + 1e-30f;
  if (!(dl + rb < av.reach3[N - first] * 0.99999f)) return false;
  const float4* e = av.ent3 + (int64_t)(N - first) * kAdjK * 2;
  for (int k = 0; k < kAdjK; ++k) {
    const float4 l = e[2 * k], h = e[2 * k + 1];
    const int X = f2i(h.w);
    if (X < 0) break;
    if (l.w * 0.99999f - dl > sqrtf(res.bound()) * 1.00001f + 1e-30f) break;
    if (box_d2(qx, qy, qz, l, h) <= res.bound()) descend(bv, first + X, qx, qy, qz, res);
  }
  return true;
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
