// build.hip -- target index build: the MI355X replacement of
// KDTree3f{dst, 16} (align_icp.cpp:165, kdtree.hpp:27-35).
//
// Pipeline (all on the context stream, no host round trip):
//   bbox (2 kernels) -> 30-bit Morton keys -> 4-pass LSD radix sort
//   (8,8,8,6 bits; per-block digit histograms, one scan, stable scatter with
//   wave-ballot ranking) -> gather Morton-ordered float4 points
//   (x, y, z, original-index bits) -> leaf boxes -> internal levels.
// The BVH is an implicit heap (root 1, children 2k/2k+1) over nleaves =
// next_pow2(ceil(m/16)) leaves of ~m/nleaves consecutive sorted points.
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

// ---- bounding box ------------------------------------------------------------
// AoS xyz input (the reference's Cloud3f layout); non-finite coordinates are
// ignored (fminf/fmaxf drop NaN; inf filtered explicitly).
__global__ __launch_bounds__(kBS) void k_bbox_partial(const float* __restrict__ xyz,
                                                      int64_t m,
                                                      float* __restrict__ part) {
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
  float mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * kBS) {
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (__builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z)) {
      mn[0] = fminf(mn[0], x); mx[0] = fmaxf(mx[0], x);
      mn[1] = fminf(mn[1], y); mx[1] = fmaxf(mx[1], y);
      mn[2] = fminf(mn[2], z); mx[2] = fmaxf(mx[2], z);
    }
  }
  __shared__ float s[kBS / kWave][6];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float v[6];
  for (int d = 0; d < 3; ++d) {
    v[d] = wave_min(mn[d]);
    v[3 + d] = wave_max(mx[d]);
  }
  if (lane == 0)
    for (int d = 0; d < 6; ++d) s[w][d] = v[d];
  __syncthreads();
  if (threadIdx.x < 6) {
    const int d = threadIdx.x;
    float r = s[0][d];
    for (int k = 1; k < kBS / kWave; ++k)
      r = d < 3 ? fminf(r, s[k][d]) : fmaxf(r, s[k][d]);
    part[blockIdx.x * 6 + d] = r;
  }
}

__global__ __launch_bounds__(kBS) void k_bbox_final(const float* __restrict__ part,
                                                    int nparts,
                                                    float* __restrict__ bbox) {
  __shared__ float s[kBS][6];
  float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = threadIdx.x; i < nparts; i += kBS)
    for (int d = 0; d < 6; ++d)
      v[d] = d < 3 ? fminf(v[d], part[i * 6 + d]) : fmaxf(v[d], part[i * 6 + d]);
  for (int d = 0; d < 6; ++d) s[threadIdx.x][d] = v[d];
  __syncthreads();
  for (int st = kBS / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st)
      for (int d = 0; d < 6; ++d)
        s[threadIdx.x][d] = d < 3 ? fminf(s[threadIdx.x][d], s[threadIdx.x + st][d])
                                  : fmaxf(s[threadIdx.x][d], s[threadIdx.x + st][d]);
    __syncthreads();
  }
  if (threadIdx.x < 6) bbox[threadIdx.x] = s[0][threadIdx.x];
}

// ---- Morton keys ---------------------------------------------------------------
__global__ __launch_bounds__(kBS) void k_morton(const float* __restrict__ xyz,
                                                int64_t m,
                                                const float* __restrict__ bbox,
                                                uint32_t* __restrict__ keys,
                                                uint32_t* __restrict__ vals) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= m) return;
  keys[i] = morton_code(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], bbox);
  vals[i] = (uint32_t)i;
}

// ---- LSD radix sort (8-bit digits, stable) ---------------------------------------
constexpr int kRsItems = 8;
constexpr int kRsTile = kBS * kRsItems;

__global__ __launch_bounds__(kBS) void k_rs_hist(const uint32_t* __restrict__ keys,
                                                 int64_t n, int shift,
                                                 uint32_t mask, int nblocks,
                                                 uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
#pragma unroll
  for (int r = 0; r < kRsItems; ++r) {
    const int64_t i = base + r * kBS + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & mask], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// ---- device-wide int32 scans (add or max; inclusive or exclusive) ----------------
// Three launches: per-tile scan (1024 items, 4 per thread) + tile totals;
// one block scans the totals (any count, 256 at a time with a carry); every
// tile then folds in its prefix.
constexpr int kScanItems = 4;
constexpr int kScanTile = kBS * kScanItems;

template <bool Max>
__device__ __forceinline__ int32_t sop(int32_t a, int32_t b) {
  return Max ? (a > b ? a : b) : a + b;
}

template <bool Max, bool Excl>
// (in may equal out: in-place scans, so no __restrict__ on either)
__global__ __launch_bounds__(kBS) void k_scan_tile(const int32_t* in, int32_t* out, int64_t n,
                                                   int32_t* __restrict__ tot) {
  __shared__ int32_t sh[kBS];
  const int32_t ident = Max ? INT32_MIN : 0;
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int32_t v[kScanItems];
  int32_t acc = ident;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = base + k < n ? in[base + k] : ident;
    acc = sop<Max>(acc, v[k]);
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 1; off < kBS; off <<= 1) {
    const int32_t o = threadIdx.x >= off ? sh[threadIdx.x - off] : ident;
    __syncthreads();
    sh[threadIdx.x] = sop<Max>(sh[threadIdx.x], o);
    __syncthreads();
  }
  int32_t run = threadIdx.x > 0 ? sh[threadIdx.x - 1] : ident;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int32_t before = run;
    run = sop<Max>(run, v[k]);
    if (base + k < n) out[base + k] = Excl ? before : run;
  }
  if (threadIdx.x == kBS - 1) tot[blockIdx.x] = sh[kBS - 1];
}

// exclusive prefix of the tile totals, in place
template <bool Max>
__global__ __launch_bounds__(kBS) void k_scan_top(int32_t* __restrict__ tot, int ntiles) {
  __shared__ int32_t sh[kBS];
  const int32_t ident = Max ? INT32_MIN : 0;
  int32_t carry = ident;
  for (int c = 0; c < ntiles; c += kBS) {
    const int i = c + threadIdx.x;
    const int32_t x = i < ntiles ? tot[i] : ident;
    sh[threadIdx.x] = x;
    __syncthreads();
    for (int off = 1; off < kBS; off <<= 1) {
      const int32_t o = threadIdx.x >= off ? sh[threadIdx.x - off] : ident;
      __syncthreads();
      sh[threadIdx.x] = sop<Max>(sh[threadIdx.x], o);
      __syncthreads();
    }
    const int32_t excl = threadIdx.x > 0 ? sh[threadIdx.x - 1] : ident;
    if (i < ntiles) tot[i] = sop<Max>(carry, excl);
    carry = sop<Max>(carry, sh[kBS - 1]);
    __syncthreads();
  }
}

template <bool Max>
__global__ __launch_bounds__(kBS) void k_scan_fix(int32_t* __restrict__ out, int64_t n,
                                                  const int32_t* __restrict__ tot) {
  if (blockIdx.x == 0) return;
  const int32_t p = tot[blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) out[base + k] = sop<Max>(p, out[base + k]);
}

__global__ __launch_bounds__(kBS) void k_rs_scatter(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n,
    int shift, uint32_t mask, int nblocks, const uint32_t* __restrict__ hist) {
  __shared__ uint32_t base[256];
  __shared__ uint32_t wcnt[kBS / kWave][257];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  base[threadIdx.x] = hist[(int64_t)threadIdx.x * nblocks + blockIdx.x];
  for (int k = 0; k < kBS / kWave; ++k) wcnt[k][threadIdx.x] = 0;
  if (threadIdx.x == 0)
    for (int k = 0; k < kBS / kWave; ++k) wcnt[k][256] = 0;
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile = (int64_t)blockIdx.x * kRsTile;
  for (int r = 0; r < kRsItems; ++r) {
    const int64_t i = tile + r * kBS + threadIdx.x;
    const bool valid = i < n;
    const uint32_t key = valid ? kin[i] : 0u;
    const uint32_t val = valid ? vin[i] : 0u;
    const uint32_t d = valid ? ((key >> shift) & mask) : 256u;
    // lanes of this wave holding the same digit (9-bit match incl. sentinel)
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      peers &= bit ? bal : ~bal;
    }
    const uint32_t rank = __popcll(peers & lt);
    const int leader = 63 - __clzll(peers);
    if (lane == leader) wcnt[w][d] = __popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t off = 0;
      for (int k = 0; k < w; ++k) off += wcnt[k][d];
      const uint32_t pos = base[d] + off + rank;
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    {
      const int dd = threadIdx.x;
      uint32_t tot = 0;
      for (int k = 0; k < kBS / kWave; ++k) {
        tot += wcnt[k][dd];
        wcnt[k][dd] = 0;
      }
      base[dd] += tot;
      if (threadIdx.x == 0)
        for (int k = 0; k < kBS / kWave; ++k) wcnt[k][256] = 0;
    }
    __syncthreads();
  }
}

// ---- sorted points + BVH -------------------------------------------------------
__global__ __launch_bounds__(kBS) void k_gather(const float* __restrict__ xyz,
                                                const uint32_t* __restrict__ perm,
                                                int64_t m, float4* __restrict__ pts) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= m) return;
  const uint32_t j = perm[i];
  pts[i] = make_float4(xyz[3 * (int64_t)j], xyz[3 * (int64_t)j + 1],
                       xyz[3 * (int64_t)j + 2], __int_as_float((int)j));
}

// inverse permutation: inv[original index] = sorted position
__global__ __launch_bounds__(kBS) void k_inverse(const uint32_t* __restrict__ perm, int64_t m,
                                                 int32_t* __restrict__ inv) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i < m) inv[perm[i]] = (int32_t)i;
}

// sorted position of original index 0 (the reference's dst.GetPoint(0)
// when nanoflann returns no neighbour)
__global__ __launch_bounds__(kBS) void k_find_pos0(const uint32_t* __restrict__ perm, int64_t m,
                                                   int32_t* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i < m && perm[i] == 0u) *out = (int32_t)i;
}

__global__ __launch_bounds__(kBS) void k_leaf_boxes(BvhView bv, float4* __restrict__ nodes) {
  const int L = blockIdx.x * kBS + threadIdx.x;
  if (L < bv.nleaves) make_leaf(bv, nodes, L);
}

// ---- compact leaves (rst_bvh.hpp leaf_cut) ---------------------------------------
// seg[i] = i where i starts a block of the code grid, else -1 (then a max
// scan turns it into each point's block start)
__global__ __launch_bounds__(kBS) void k_leaf_seg(const uint32_t* __restrict__ codes, int64_t m,
                                                  int32_t* __restrict__ seg) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= m) return;
  seg[i] = (i == 0 || (codes[i] >> kLeafCellShift) != (codes[i - 1] >> kLeafCellShift)) ? (int)i
                                                                                         : -1;
}

__global__ __launch_bounds__(kBS) void k_leaf_cutflag(const uint32_t* __restrict__ codes,
                                                      const int32_t* __restrict__ seg, int64_t m,
                                                      int32_t* __restrict__ cut) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= m) return;
  cut[i] = leaf_cut(codes, (int)i, seg[i]) ? 1 : 0;
}

// the cut positions (where the inclusive count of cuts steps) are the leaf
// starts.  Read-only over the counts: thread i reads entry i - 1, so the
// counts -> leaf ids rewrite (k_leaf_ids) must be a separate launch (a
// wavefront writing entry i - 1 first made leaf starts vanish at random --
// leaves of up to 31 points)
__global__ __launch_bounds__(kBS) void k_leaf_start(const int32_t* __restrict__ pleaf, int64_t m,
                                                    int32_t* __restrict__ lstart) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= m) return;
  const int32_t c = pleaf[i];
  if (i == 0 || pleaf[i - 1] != c) lstart[c - 1] = (int32_t)i;
}

// pleaf = inclusive count of cuts - 1
__global__ __launch_bounds__(kBS) void k_leaf_ids(int32_t* __restrict__ pleaf, int64_t m) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i < m) pleaf[i] -= 1;
}

__global__ __launch_bounds__(kBS) void k_leaf_tail(int32_t* __restrict__ lstart, int nl0, int nl,
                                                   int32_t m) {
  const int L = nl0 + blockIdx.x * kBS + threadIdx.x;
  if (L <= nl) lstart[L] = m;
}

// leaf adjacency (the tracking index, rst_bvh.hpp): one wavefront per leaf
__global__ __launch_bounds__(kBS) void k_leaf_adj(BvhView bv, int first, float4* __restrict__ ent,
                                                  float* __restrict__ reach) {
  __shared__ WnnScratch wsc[kBS / kWave];
  const int L = blockIdx.x * (kBS / kWave) + threadIdx.x / kWave;
  if (L < first) leaf_adj_wave(bv, first, L, ent, reach, wsc[threadIdx.x / kWave]);
}

__global__ __launch_bounds__(kBS) void k_level(float4* __restrict__ nodes, int lo_k,
                                               int count) {
  const int i = blockIdx.x * kBS + threadIdx.x;
  if (i < count) make_internal(nodes, lo_k + i);
}

// all levels with fewer than 2*kBS nodes, one block, barrier per level
__global__ __launch_bounds__(kBS) void k_levels_top(float4* __restrict__ nodes,
                                                    int top_count) {
  for (int cnt = top_count; cnt >= 1; cnt >>= 1) {
    for (int i = threadIdx.x; i < cnt; i += kBS) make_internal(nodes, cnt + i);
    __syncthreads();
  }
}

inline int blocks_for(int64_t n, int per = kBS) {
  return (int)std::max<int64_t>(1, (n + per - 1) / per);
}

}  // namespace

template <bool Max, bool Excl>
void scan_i32(hipStream_t st, const int32_t* in, int32_t* out, int64_t n, int32_t* tot) {
  const int nt = (int)std::max<int64_t>(1, (n + kScanTile - 1) / kScanTile);
  k_scan_tile<Max, Excl><<<nt, kBS, 0, st>>>(in, out, n, tot);
  k_scan_top<Max><<<1, kBS, 0, st>>>(tot, nt);
  k_scan_fix<Max><<<nt, kBS, 0, st>>>(out, n, tot);
}

int radix_sort_pairs(rst_ctx* ctx, uint32_t* keys, uint32_t* vals, uint32_t* ktmp,
                     uint32_t* vtmp, uint32_t* hist, int32_t* stot, int64_t n) {
  hipStream_t st = ctx->stream;
  const int nb = blocks_for(n, kRsTile);
  const int shifts[4] = {0, 8, 16, 24};
  const uint32_t masks[4] = {0xff, 0xff, 0xff, 0x3f};
  uint32_t *ka = keys, *va = vals, *kb = ktmp, *vb = vtmp;
  for (int p = 0; p < 4; ++p) {
    k_rs_hist<<<nb, kBS, 0, st>>>(ka, n, shifts[p], masks[p], nb, hist);
    scan_i32<false, true>(st, (const int32_t*)hist, (int32_t*)hist, (int64_t)256 * nb, stot);
    k_rs_scatter<<<nb, kBS, 0, st>>>(ka, va, kb, vb, n, shifts[p], masks[p], nb, hist);
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  RST_HIP(hipGetLastError());
  return RST_OK;  // 4 passes: result back in keys/vals
}

AdjView adj_of(const rst_target* t) {
  AdjView a;
  a.ent = t->adj;
  a.ent2 = t->adj2;
  a.reach2 = t->reach2;
  a.ent3 = t->adj3;
  a.reach3 = t->reach3;
  a.reach = t->reach;
  return a;
}

size_t target_index_bytes(const rst_target* t) {
  if (!t->has_bvh) return 0;
  return (size_t)4 * t->nleaves * sizeof(float4);
}

BvhView view_of(const rst_target* t) {
  BvhView v;
  v.pts = t->pts;
  v.nodes = t->nodes;
  v.lstart = t->lstart;
  v.pleaf = t->pleaf;
  v.codes = t->codes;
  v.bbox = t->codes ? (const float*)(t->codes + std::max<int64_t>(t->m, 1)) : nullptr;
  v.m = (int32_t)t->m;
  v.nleaves = t->nleaves;
  v.lg = t->lg;
  v.pad = 0;
  return v;
}

int target_build_device(rst_ctx* ctx, const float* d_xyz, int64_t m, bool with_bvh,
                        rst_target** out) {
  if (!ctx || !out || m < 0 || (m > 0 && !d_xyz)) return RST_E_ARG;
  // leaf-range tags of the adjacency pack begin * 32 (rst_bvh.hpp leaf_tag)
  if (m >= (int64_t)1 << 26) return RST_E_ARG;
  rst_target* t = new rst_target();
  t->ctx = ctx;
  t->m = m;
  {
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    ctx->live.push_back(t);
  }
  hipStream_t st = ctx->stream;
  const int64_t mp = std::max<int64_t>(m, 1);
  auto ta = [&](auto** p, size_t bytes) { return target_alloc(t, bytes, (void**)p) >= 0; };
  if (!ta(&t->pts, sizeof(float4) * (mp + kPtsPad)) || !ta(&t->inv, sizeof(int32_t) * mp) ||
      !ta(&t->pleaf, sizeof(int32_t) * mp) ||
      !ta(&t->codes, sizeof(uint32_t) * mp + sizeof(float) * 8)) {
    rst_target_free(t);
    return RST_E_NOMEM;
  }
  // leaves: how many is known only after the sort (an empty cloud: one
  // empty leaf)
  auto alloc_tree = [&](int64_t NL) -> int {
    int64_t nl = 1;
    int lg = 0;
    while (nl < NL) {
      nl <<= 1;
      ++lg;
    }
    t->nleaves = (int32_t)nl;
    t->lg = lg;
    const int64_t n2 = std::max<int64_t>(nl >> kAdj2Shift, 1);
    const int64_t n3 = std::max<int64_t>(nl >> kAdj3Shift, 1);
    if (!ta(&t->nodes, sizeof(float4) * 4 * nl) || !ta(&t->lstart, sizeof(int32_t) * (nl + 1)) ||
        !ta(&t->adj, sizeof(float4) * 2 * kAdjK * nl) || !ta(&t->reach, sizeof(float) * nl) ||
        !ta(&t->adj2, sizeof(float4) * 2 * kAdjK * n2) || !ta(&t->reach2, sizeof(float) * n2) ||
        !ta(&t->adj3, sizeof(float4) * 2 * kAdjK * n3) || !ta(&t->reach3, sizeof(float) * n3))
      return RST_E_NOMEM;
    if (nl < (1 << kAdj2Shift) && hipMemsetAsync(t->reach2, 0, sizeof(float), st) != hipSuccess)
      return RST_E_HIP;
    if (nl < (1 << kAdj3Shift) && hipMemsetAsync(t->reach3, 0, sizeof(float), st) != hipSuccess)
      return RST_E_HIP;
    t->has_bvh = true;
    return RST_OK;
  };
  if (m == 0) {
    int s = with_bvh ? alloc_tree(1) : RST_OK;
    if (s >= 0 && with_bvh) {
      // one empty leaf: lstart = {0, 0}, empty box, no adjacency
      const float4 e[2] = {make_float4(INFINITY, INFINITY, INFINITY, 0.f),
                           make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f)};
      const int32_t z[2] = {0, 0};
      if (hipMemcpyAsync(t->nodes + 2, e, sizeof(e), hipMemcpyHostToDevice, st) != hipSuccess ||
          hipMemcpyAsync(t->lstart, z, sizeof(z), hipMemcpyHostToDevice, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        s = RST_E_HIP;
    }
    if (s < 0) {
      rst_target_free(t);
      return s;
    }
    *out = t;
    return RST_OK;
  }
  // workspace: bbox partials | bbox | keys | vals | ktmp | vtmp | hist | scan tiles
  const int nbb = std::min(1024, blocks_for(m));
  const int nb = blocks_for(m, kRsTile);
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_part = carve(sizeof(float) * 6 * nbb);
  const size_t o_bbox = carve(sizeof(float) * 8);
  const size_t o_k = carve(sizeof(uint32_t) * m);
  const size_t o_v = carve(sizeof(uint32_t) * m);
  const size_t o_kt = carve(sizeof(uint32_t) * m);
  const size_t o_vt = carve(sizeof(uint32_t) * m);
  const size_t o_h = carve(sizeof(uint32_t) * 256 * (size_t)nb);
  const size_t o_tot = carve(sizeof(int32_t) * (256 * (size_t)nb / kScanTile + m / kScanTile + 64));
  void* ws = nullptr;
  int s = ctx_workspace(ctx, off, &ws);
  if (s < 0) {
    rst_target_free(t);
    return s;
  }
  char* w = (char*)ws;
  float* part = (float*)(w + o_part);
  float* bbox = (float*)(w + o_bbox);
  uint32_t* keys = (uint32_t*)(w + o_k);
  uint32_t* vals = (uint32_t*)(w + o_v);
  int32_t* tot = (int32_t*)(w + o_tot);
  k_bbox_partial<<<nbb, kBS, 0, st>>>(d_xyz, m, part);
  k_bbox_final<<<1, kBS, 0, st>>>(part, nbb, bbox);
  k_morton<<<blocks_for(m), kBS, 0, st>>>(d_xyz, m, bbox, keys, vals);
  s = radix_sort_pairs(ctx, keys, vals, (uint32_t*)(w + o_kt), (uint32_t*)(w + o_vt),
                       (uint32_t*)(w + o_h), tot, m);
  if (s < 0) {
    rst_target_free(t);
    return s;
  }
  // sorted codes + their box stay with the target (cold-start seeds)
  if (hipMemcpyAsync(t->codes, keys, sizeof(uint32_t) * m, hipMemcpyDeviceToDevice, st) !=
          hipSuccess ||
      hipMemcpyAsync(t->codes + mp, bbox, sizeof(float) * 6, hipMemcpyDeviceToDevice, st) !=
          hipSuccess) {
    rst_target_free(t);
    return RST_E_HIP;
  }
  k_gather<<<blocks_for(m), kBS, 0, st>>>(d_xyz, vals, m, t->pts);
  k_find_pos0<<<blocks_for(m), kBS, 0, st>>>(vals, m, (int32_t*)(bbox + 6));
  k_inverse<<<blocks_for(m), kBS, 0, st>>>(vals, m, t->inv);
  int32_t NL = 0;
  if (with_bvh) {
    // compact leaves: block starts (max scan), cut flags, leaf ids (add scan)
    int32_t* seg = (int32_t*)(w + o_kt);
    k_leaf_seg<<<blocks_for(m), kBS, 0, st>>>(t->codes, m, seg);
    scan_i32<true, false>(st, seg, seg, m, tot);
    k_leaf_cutflag<<<blocks_for(m), kBS, 0, st>>>(t->codes, seg, m, t->pleaf);
    scan_i32<false, false>(st, t->pleaf, t->pleaf, m, tot);
    if (hipMemcpyAsync(&NL, t->pleaf + (m - 1), sizeof(int32_t), hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      rst_target_free(t);
      return RST_E_HIP;
    }
    s = alloc_tree(std::max<int32_t>(NL, 1));
    if (s < 0) {
      rst_target_free(t);
      return s;
    }
    const int nl = t->nleaves;
    k_leaf_start<<<blocks_for(m), kBS, 0, st>>>(t->pleaf, m, t->lstart);
    k_leaf_ids<<<blocks_for(m), kBS, 0, st>>>(t->pleaf, m);
    k_leaf_tail<<<blocks_for(nl + 1 - NL), kBS, 0, st>>>(t->lstart, NL, nl, (int32_t)m);
    k_leaf_boxes<<<blocks_for(nl), kBS, 0, st>>>(view_of(t), t->nodes);
    int64_t cnt = nl / 2;
    while (cnt >= 2 * kBS) {
      k_level<<<blocks_for(cnt), kBS, 0, st>>>(t->nodes, (int)cnt, (int)cnt);
      cnt >>= 1;
    }
    if (cnt >= 1) k_levels_top<<<1, kBS, 0, st>>>(t->nodes, (int)cnt);
    k_leaf_adj<<<blocks_for(nl, kBS / kWave), kBS, 0, st>>>(view_of(t), nl, t->adj, t->reach);
    if (nl >= (1 << kAdj2Shift))
      k_leaf_adj<<<blocks_for(nl >> kAdj2Shift, kBS / kWave), kBS, 0, st>>>(
          view_of(t), nl >> kAdj2Shift, t->adj2, t->reach2);
    if (nl >= (1 << kAdj3Shift))
      k_leaf_adj<<<blocks_for(nl >> kAdj3Shift, kBS / kWave), kBS, 0, st>>>(
          view_of(t), nl >> kAdj3Shift, t->adj3, t->reach3);
  }
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(t->bbox, bbox, sizeof(float) * 6, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(&t->pos0, bbox + 6, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    rst_target_free(t);
    return RST_E_HIP;
  }
  *out = t;
  return RST_OK;
}

}  // namespace rst
