// voxel.hip -- the preprocessing every reference caller runs right before
// AlignIcp3d (rs_replay_app.cpp:229,246-247,
// rs_align_app.cpp:254-255):
//
//   RemoveNans      (point_cloud_utils.cpp:163-174): drop points with a
//                   non-finite coordinate, order kept;
//   DownsampleVoxel (point_cloud_utils.cpp:34-68): one point per voxel
//                   floor(p / voxel_size) -- the FIRST point (lowest index)
//                   of each voxel, since the reference emplaces only when the
//                   key is new -- emitted in the reference's order, its
//                   std::unordered_map's iteration (k_umap_order).  The voxel key is
//                   (int)floorf(p / v) per axis; a NaN / out-of-int-range
//                   value maps to INT_MIN, what x86-64's cvttss2si yields
//                   for the reference's cast (so NaN points share one voxel).
//
// Both are order-preserving GPU compactions: per-tile counts, one scan,
// ballot-ranked writes (as unproject.hip).  The voxel filter first claims
// one hash-table slot per voxel (lock-free open addressing; slot equality is
// tested on the representative point's own key, so keys need no packing),
// then takes the minimum index per slot with atomicMin, then keeps point i
// iff it is its slot's minimum.  HBM traffic: 12 B/pt in (+12 B/pt per
// probe), 12 B/kept pt out, 8 B/slot of table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <unordered_map>  // (libstdc++'s _Prime_rehash_policy: umap_schedule)

#include "rst_device.hpp"
#include "rst_internal.hpp"

namespace rst {
namespace {

constexpr int kBS = 256;
constexpr int kRounds = 4;
constexpr int kTile = kBS * kRounds;
constexpr int32_t kEmptySlot = -1;

__device__ __forceinline__ bool finite_pt(const float* __restrict__ xyz, int64_t i) {
  return __builtin_isfinite(xyz[3 * i]) && __builtin_isfinite(xyz[3 * i + 1]) &&
         __builtin_isfinite(xyz[3 * i + 2]);
}

// Voxel keys with x86-64 cvttss2si semantics outside int range / NaN:
//   kind 0 (DownsampleVoxel, point_cloud_utils.cpp:41-42): (int)floor(x / v);
//   kind 1 (CloudAccumulator::GetVoxelIndex, rs_replay_app.cpp:108-110):
//           (int)(x * v), v = the float inverse voxel size (truncation).
__device__ __forceinline__ int vox_coord(float x, float v, int kind) {
  const float q = kind == 0 ? floorf(x / v) : x * v;
  return (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT_MIN;
}

struct Vox {
  int x, y, z;
};

__device__ __forceinline__ Vox vox_of(const float* __restrict__ xyz, int64_t i, float v,
                                      int kind = 0) {
  return Vox{vox_coord(xyz[3 * i], v, kind), vox_coord(xyz[3 * i + 1], v, kind),
             vox_coord(xyz[3 * i + 2], v, kind)};
}

__device__ __forceinline__ uint32_t vox_hash(const Vox& k) {
  uint32_t h = (uint32_t)k.x * 0x9E3779B1u;
  h ^= (uint32_t)k.y * 0x85EBCA77u + (h << 6) + (h >> 2);
  h ^= (uint32_t)k.z * 0xC2B2AE3Du + (h << 6) + (h >> 2);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

// ---- order-preserving compaction (count / scan / write) ------------------------
// mode 0 = RemoveNans (keep finite points), 1 = keep flagged points
__device__ __forceinline__ bool keep_pt(int mode, const float* __restrict__ xyz,
                                        const uint8_t* __restrict__ flag, int64_t i) {
  return mode == 0 ? finite_pt(xyz, i) : flag[i] != 0;
}

__global__ __launch_bounds__(kBS) void k_keep_count(const float* __restrict__ xyz, int64_t n,
                                                    int mode, const uint8_t* __restrict__ flag,
                                                    uint32_t* __restrict__ counts) {
  __shared__ uint32_t s[kBS / kWave];
  uint32_t cnt = 0;
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t i = base + r * kBS + threadIdx.x;
    if (i < n && keep_pt(mode, xyz, flag, i)) ++cnt;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, kWave);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < kBS / kWave; ++k) t += s[k];
    counts[blockIdx.x] = t;
  }
}

// exclusive scan of the tile counts in one block
__global__ __launch_bounds__(1024) void k_scan_counts(uint32_t* __restrict__ a, int n,
                                                      uint32_t* __restrict__ total) {
  __shared__ uint32_t s[1024];
  const int per = (n + 1023) / 1024;
  const int b = threadIdx.x * per;
  const int e = min(b + per, n);
  uint32_t sum = 0;
  for (int i = b; i < e; ++i) sum += a[i];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = threadIdx.x >= off ? s[threadIdx.x - off] : 0u;
    __syncthreads();
    s[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - sum;
  for (int i = b; i < e; ++i) {
    const uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
  if (threadIdx.x == 1023) *total = s[1023];
}

__global__ __launch_bounds__(kBS) void k_keep_write(const float* __restrict__ xyz, int64_t n,
                                                    int mode, const uint8_t* __restrict__ flag,
                                                    const uint32_t* __restrict__ offsets,
                                                    float* __restrict__ out) {
  __shared__ uint32_t wtot[kBS / kWave];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t run = offsets[blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * kTile;
  for (int r = 0; r < kRounds; ++r) {
    const int64_t i = base + r * kBS + threadIdx.x;
    const bool ok = i < n && keep_pt(mode, xyz, flag, i);
    const uint64_t bal = __ballot(ok);
    if (lane == 0) wtot[w] = __popcll(bal);
    __syncthreads();
    uint32_t off = run;
    for (int k = 0; k < w; ++k) off += wtot[k];
    if (ok) {
      const int64_t o = off + __popcll(bal & lt);
      out[3 * o + 0] = xyz[3 * i + 0];
      out[3 * o + 1] = xyz[3 * i + 1];
      out[3 * o + 2] = xyz[3 * i + 2];
    }
    uint32_t tot = 0;
    for (int k = 0; k < kBS / kWave; ++k) tot += wtot[k];
    run += tot;
    __syncthreads();
  }
}

// ---- voxel table ---------------------------------------------------------------------
// 1. claim the slot of i's voxel: the first empty slot on its probe sequence
//    (CAS), or the slot whose representative point lies in the same voxel
__global__ __launch_bounds__(kBS) void k_vox_claim(const float* __restrict__ xyz, int64_t n,
                                                   float v, int kind, int32_t* __restrict__ rep,
                                                   uint32_t mask, int32_t* __restrict__ slot_of) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  const Vox k = vox_of(xyz, i, v, kind);
  uint32_t h = vox_hash(k) & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    int32_t cur = __hip_atomic_load(&rep[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == kEmptySlot) {
      const int32_t prev = atomicCAS(&rep[h], kEmptySlot, (int32_t)i);
      if (prev == kEmptySlot) {
        slot_of[i] = (int32_t)h;
        return;
      }
      cur = prev;
    }
    const Vox o = vox_of(xyz, cur, v, kind);
    if (o.x == k.x && o.y == k.y && o.z == k.z) {
      slot_of[i] = (int32_t)h;
      return;
    }
    h = (h + 1) & mask;
  }
  slot_of[i] = -1;  // unreachable: the table has more slots than points
}

// 2. the first (lowest-index) point of each voxel
__global__ __launch_bounds__(kBS) void k_vox_min(int64_t n, const int32_t* __restrict__ slot_of,
                                                 int32_t* __restrict__ minidx) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slot_of[i];
  if (s >= 0) atomicMin(&minidx[s], (int32_t)i);
}

// 3. keep point i iff it is its voxel's first
__global__ __launch_bounds__(kBS) void k_vox_flag(int64_t n, const int32_t* __restrict__ slot_of,
                                                  const int32_t* __restrict__ minidx,
                                                  uint8_t* __restrict__ flag) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slot_of[i];
  flag[i] = (s >= 0 && minidx[s] == (int32_t)i) ? 1 : 0;
}

inline int blocks_for(int64_t n, int per = kBS) {
  return (int)std::max<int64_t>(1, (n + per - 1) / per);
}

int compact(rst_ctx* ctx, const float* d_xyz, int64_t n, int mode, const uint8_t* d_flag,
            uint32_t* counts, uint32_t* total, float* d_out, int64_t* n_out) {
  hipStream_t st = ctx->stream;
  const int nb = blocks_for(n, kTile);
  k_keep_count<<<nb, kBS, 0, st>>>(d_xyz, n, mode, d_flag, counts);
  k_scan_counts<<<1, 1024, 0, st>>>(counts, nb, total);
  k_keep_write<<<nb, kBS, 0, st>>>(d_xyz, n, mode, d_flag, counts, d_out);
  RST_HIP(hipGetLastError());
  uint32_t h = 0;
  RST_HIP(hipMemcpyAsync(&h, total, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  *n_out = h;
  return RST_OK;
}

// ---- the reference's std::unordered_map iteration order ------------------------------
// DownsampleVoxel (point_cloud_utils.cpp:54-57,63-66) and
// CloudAccumulator::ExtractPointCloud (rs_replay_app.cpp:112-121) emit their
// points by iterating a std::unordered_map that received the distinct voxel
// keys in input order (find, then emplace).  libstdc++'s table keeps one
// singly-linked list: an insert into an empty bucket goes to the list's
// front, any other to the front of its bucket's run; a rehash walks the old
// list and re-inserts each node the same way.  So between rehashes the list
// is one run per bucket, the bucket created later first, the later arrival
// first inside a bucket, and at every level the order sorts by (creation of
// the element's bucket, arrival), both descending -- arrival being the
// element's position in the list the last rehash walked, or its insertion
// index when it came after it.  k_umap_order replays that level by level
// from the container's rehash schedule (umap_schedule: libstdc++'s own
// _Prime_rehash_policy), with no list: per level the buckets' creation times
// (atomicMin of arrival), their sizes, one suffix scan over arrivals for the
// runs' starts, and each bucket's members ranked by arrival.  The hash is
// the reference's boost::hash_combine over std::hash<int> / hash_value(int)
// (both size_t(k)), Boost <= 1.80's classic form (oracle/rst_oracle_umap.cpp
// pins the model against a real std::unordered_map, tests/test_oracle.py).
constexpr int kUmapT = 1024;
constexpr int kUmapIl = 4;  // elements per thread with their loads interleaved
constexpr int kUmapMaxLevels = 48;
struct UmapSched {
  int nl;
  int64_t r[kUmapMaxLevels];  // elements before the insert that rehashed
  int64_t B[kUmapMaxLevels];  // the bucket count it rehashed to
};

__device__ __forceinline__ uint64_t boost_combine3(const Vox& k) {
  uint64_t seed = 0;
  const int v[3] = {k.x, k.y, k.z};
#pragma unroll
  for (int i = 0; i < 3; ++i) seed ^= (uint64_t)(int64_t)v[i] + 0x9e3779b9ull + (seed << 6) + (seed >> 2);
  return seed;
}

// cross-wave reads of the scratch arrays at agent scope: some are written by
// atomics, which act in L2 (no stale vL1 line is ever read)
template <class T>
__device__ __forceinline__ T ld(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one workgroup: exclusive scan of a[0, n) in place (forward) or the suffix
// form s[i] = sum of a[j > i] (backward); returns the total
__device__ int64_t wg_scan(int32_t* a, int64_t n, bool suffix, int64_t* part) {
  const int t = threadIdx.x;
  const int64_t per = (n + kUmapT - 1) / kUmapT;
  const int64_t b0 = t * per, b1 = min(n, b0 + per);
  int64_t sum = 0;
  for (int64_t i = b0; i < b1; ++i) sum += ld(a + (suffix ? n - 1 - i : i));
  // the partials' exclusive scan: wave-level shuffles, then the 16 wave
  // totals (r10a: one thread walking the 1024 partials took ~25 us per scan,
  // two scans per rehash level -- k_umap_order ~0.9 ms a call at 15k keys)
  const int lane = t & (kWave - 1), wv = t / kWave;
  int64_t inc = sum;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int64_t y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  if (lane == kWave - 1) part[wv] = inc;
  __syncthreads();
  if (t == 0) {
    int64_t run = 0;
    for (int k = 0; k < kUmapT / kWave; ++k) {
      const int64_t v = part[k];
      part[k] = run;
      run += v;
    }
    part[kUmapT] = run;
  }
  __syncthreads();
  int64_t run = part[wv] + inc - sum;
  for (int64_t i = b0; i < b1; ++i) {
    const int64_t j = suffix ? n - 1 - i : i;
    const int32_t v = ld(a + j);
    __hip_atomic_store(a + j, (int32_t)run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    run += v;
  }
  const int64_t tot = part[kUmapT];
  __syncthreads();
  return tot;
}

struct UmapWs {
  uint64_t* h;
  int32_t *pos, *arr, *bk, *mem, *hs;     // [n]
  int32_t *ctime, *cnt, *start, *fill;  // [B max]
};

__global__ __launch_bounds__(kUmapT) void k_umap_order(const float* __restrict__ pts, int64_t n, float v,
                                                       int kind, UmapSched sc, UmapWs w,
                                                       float* __restrict__ out) {
  __shared__ int64_t part[kUmapT + 1];
  const int t = threadIdx.x;
  auto st = [](int32_t* p, int32_t x) { __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int64_t e = t; e < n; e += kUmapT) w.h[e] = boost_combine3(vox_of(pts, e, v, kind));
  __syncthreads();
  for (int l = 0; l < sc.nl; ++l) {
    const int64_t r = sc.r[l], B = sc.B[l];
    const int64_t nl = l + 1 < sc.nl ? sc.r[l + 1] : n;
    for (int64_t b = t; b < B; b += kUmapT) {
      st(w.ctime + b, INT_MAX);
      st(w.cnt + b, 0);
      st(w.fill + b, 0);
    }
    for (int64_t a = t; a < nl; a += kUmapT) st(w.hs + a, 0);
    __syncthreads();
    // arrival (the walked list's position, or the insertion index), bucket
    for (int64_t e = t; e < nl; e += kUmapT) {
      const int32_t a = e < r ? ld(w.pos + e) : (int32_t)e;
      const int32_t b = (int32_t)(ld(w.h + e) % (uint64_t)B);
      st(w.arr + e, a);
      st(w.bk + e, b);
      atomicMin(w.ctime + b, a);
      atomicAdd(w.cnt + b, 1);
    }
    __syncthreads();
    // the buckets' member ranges, and each bucket's size at its creation's arrival
    for (int64_t b = t; b < B; b += kUmapT) st(w.start + b, ld(w.cnt + b));
    __syncthreads();
    wg_scan(w.start, B, false, part);
    for (int64_t e0 = t; e0 < nl; e0 += (int64_t)kUmapIl * kUmapT) {  // (interleaved as below)
      int32_t b[kUmapIl], a[kUmapIl], sl[kUmapIl], ct[kUmapIl], cn[kUmapIl];
#pragma unroll
      for (int u = 0; u < kUmapIl; ++u) {
        const int64_t e = e0 + (int64_t)u * kUmapT;
        b[u] = e < nl ? ld(w.bk + e) : -1;
        a[u] = e < nl ? ld(w.arr + e) : 0;
      }
#pragma unroll
      for (int u = 0; u < kUmapIl; ++u) {
        sl[u] = b[u] >= 0 ? ld(w.start + b[u]) + atomicAdd(w.fill + b[u], 1) : 0;
        ct[u] = b[u] >= 0 ? ld(w.ctime + b[u]) : -1;
        cn[u] = b[u] >= 0 ? ld(w.cnt + b[u]) : 0;
      }
#pragma unroll
      for (int u = 0; u < kUmapIl; ++u) {
        if (b[u] < 0) continue;
        st(w.mem + sl[u], (int32_t)(e0 + (int64_t)u * kUmapT));
        if (a[u] == ct[u]) st(w.hs + a[u], cn[u]);
      }
    }
    __syncthreads();
    // hs[a] = the elements of buckets created after arrival a: a run's start
    wg_scan(w.hs, nl, true, part);
    // each element's place: its bucket's run start plus the members of its
    // bucket arriving later (they come first).  Per element, kUmapIl of
    // them interleaved so their dependent loads overlap (r10b: a loop over
    // the buckets -- most empty -- walked one L2 round trip after another,
    // ~60 us a rehash level at 15k keys)
    for (int64_t e0 = t; e0 < nl; e0 += (int64_t)kUmapIl * kUmapT) {
      int32_t b[kUmapIl], a[kUmapIl], c[kUmapIl], s0[kUmapIl], ct[kUmapIl], rank[kUmapIl];
      bool ok[kUmapIl];
#pragma unroll
      for (int u = 0; u < kUmapIl; ++u) {
        const int64_t e = e0 + (int64_t)u * kUmapT;
        ok[u] = e < nl;
        b[u] = ok[u] ? ld(w.bk + e) : 0;
        a[u] = ok[u] ? ld(w.arr + e) : 0;
      }
#pragma unroll
      for (int u = 0; u < kUmapIl; ++u) {
        c[u] = ok[u] ? ld(w.cnt + b[u]) : 0;
        s0[u] = ok[u] ? ld(w.start + b[u]) : 0;
        ct[u] = ok[u] ? ld(w.ctime + b[u]) : 0;
        rank[u] = 0;
      }
      int cm = 0;
#pragma unroll
      for (int u = 0; u < kUmapIl; ++u) cm = max(cm, c[u]);
      for (int32_t j = 0; j < cm; ++j) {
        int32_t m[kUmapIl];
#pragma unroll
        for (int u = 0; u < kUmapIl; ++u) m[u] = j < c[u] ? ld(w.mem + s0[u] + j) : -1;
#pragma unroll
        for (int u = 0; u < kUmapIl; ++u) rank[u] += (m[u] >= 0 && ld(w.arr + m[u]) > a[u]) ? 1 : 0;
      }
#pragma unroll
      for (int u = 0; u < kUmapIl; ++u)
        if (ok[u]) st(w.pos + e0 + (int64_t)u * kUmapT, ld(w.hs + ct[u]) + rank[u]);
    }
    __syncthreads();
  }
  for (int64_t e = t; e < n; e += kUmapT) {
    const int64_t o = ld(w.pos + e);
    out[3 * o + 0] = pts[3 * e + 0];
    out[3 * o + 1] = pts[3 * e + 1];
    out[3 * o + 2] = pts[3 * e + 2];
  }
}

// The same replay for up to kUsMaxN keys (the reference callers' 5 cm
// clouds, ~15k voxels), on one CU from LDS: per level a counting sort of
// the elements by bucket (16-bit counts, two a word), each element's bucket
// read from the sort -- its creation time (the members' least arrival), its
// size, the element's rank (members arriving later) -- then one suffix scan
// over arrivals for the runs' starts.  Every element stays with one thread
// across the levels, its hash in registers; 11 levels at 15k keys with
// LDS atomics and scans in place of k_umap_order's global round trips
// (r10: ~570 us a call).
constexpr int kUsT = 1024;
constexpr int kUsMaxN = 16384;
constexpr int kUsPer = kUsMaxN / kUsT;  // elements a thread
constexpr int kUsMaxB = 20753;          // the schedule's last bucket count at kUsMaxN keys
struct UsLds {
  uint32_t cs[kUsMaxB / 2 + 2];  // bucket b's count, then start: half b & 1 of word b >> 1
  int16_t bk[kUsMaxN];           // the element's bucket
  int16_t arr[kUsMaxN];          // its arrival; at a level's end its place
  int16_t mem[kUsMaxN];          // the buckets' members; then a creation arrival's run start
  int part[kUsT / kWave + 1];
};
static_assert(sizeof(UsLds) <= 160 * 1024, "k_umap_small LDS");
static_assert(kUsMaxN <= 32767, "16-bit arrivals");

// exclusive scan of one int per thread over the workgroup; returns the total
__device__ __forceinline__ int us_scan(int v, int* part, int& excl) {
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  int inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  if (lane == kWave - 1) part[wv] = inc;
  __syncthreads();
  if (t < kWave) {
    const int pv = t < kUsT / kWave ? part[t] : 0;
    int pi = pv;
#pragma unroll
    for (int o = 1; o < kUsT / kWave; o <<= 1) {
      const int y = __shfl_up(pi, o, kWave);
      if (lane >= o) pi += y;
    }
    if (t < kUsT / kWave) part[t] = pi - pv;
    if (t == kUsT / kWave - 1) part[kUsT / kWave] = pi;
  }
  __syncthreads();
  excl = part[wv] + inc - v;
  const int tot = part[kUsT / kWave];
  __syncthreads();
  return tot;
}

__device__ __forceinline__ int us_get(const uint32_t* cs, int b) { return (int)((cs[b >> 1] >> (16 * (b & 1))) & 0xffffu); }

__global__ __launch_bounds__(kUsT) void k_umap_small(const float* __restrict__ pts, int n, float v, int kind,
                                                    UmapSched sc, float* __restrict__ out) {
  __shared__ UsLds W;
  const int t = threadIdx.x;
  uint64_t h[kUsPer];  // element t + j kUsT's hash
#pragma unroll
  for (int j = 0; j < kUsPer; ++j) {
    const int e = t + j * kUsT;
    h[j] = e < n ? boost_combine3(vox_of(pts, e, v, kind)) : 0;
  }
  for (int l = 0; l < sc.nl; ++l) {
    const int r = (int)sc.r[l], B = (int)sc.B[l];
    const int nl = l + 1 < sc.nl ? (int)sc.r[l + 1] : n;
    const int nw = B / 2 + 1;
    for (int k = t; k < nw; k += kUsT) W.cs[k] = 0;
    __syncthreads();
    // arrivals (the walked list's place, kept from the last level, or the
    // insertion index) and buckets; the buckets' counts
#pragma unroll
    for (int j = 0; j < kUsPer; ++j) {
      const int e = t + j * kUsT;
      if (e < nl) {
        const int b = (int)(h[j] % (uint64_t)B);
        W.bk[e] = (int16_t)b;
        if (e >= r) W.arr[e] = (int16_t)e;
        atomicAdd(&W.cs[b >> 1], 1u << (16 * (b & 1)));
      }
    }
    __syncthreads();
    // the counts -> the buckets' starts (thread t: words [t per, (t + 1) per))
    {
      const int per = (nw + kUsT - 1) / kUsT;
      const int w0 = min(nw, t * per), w1 = min(nw, w0 + per);
      int sum = 0;
      for (int k = w0; k < w1; ++k) sum += (int)(W.cs[k] & 0xffffu) + (int)(W.cs[k] >> 16);
      int run;
      us_scan(sum, W.part, run);
      for (int k = w0; k < w1; ++k) {
        const uint32_t c = W.cs[k];
        const int lo = run;
        run += (int)(c & 0xffffu);
        W.cs[k] = (uint32_t)lo | ((uint32_t)run << 16);
        run += (int)(c >> 16);
      }
    }
    __syncthreads();
    // members by bucket (each start advances to its bucket's end)
#pragma unroll
    for (int j = 0; j < kUsPer; ++j) {
      const int e = t + j * kUsT;
      if (e < nl) {
        const int b = W.bk[e];
        const uint32_t old = atomicAdd(&W.cs[b >> 1], 1u << (16 * (b & 1)));
        W.mem[(old >> (16 * (b & 1))) & 0xffffu] = (int16_t)e;
      }
    }
    __syncthreads();
    // per element: its bucket's creation, size, and the members after it
    int rk[kUsPer], ct[kUsPer], sz[kUsPer];
#pragma unroll
    for (int j = 0; j < kUsPer; ++j) {
      const int e = t + j * kUsT;
      rk[j] = 0;
      ct[j] = -1;
      sz[j] = 0;
      if (e < nl) {
        const int b = W.bk[e];
        const int end = us_get(W.cs, b), beg = b == 0 ? 0 : us_get(W.cs, b - 1);
        const int a = W.arr[e];
        int c = a, rr = 0;
        for (int k = beg; k < end; ++k) {
          const int am = W.arr[W.mem[k]];
          rr += am > a ? 1 : 0;
          c = min(c, am);
        }
        rk[j] = rr;
        ct[j] = c;
        sz[j] = end - beg;
      }
    }
    __syncthreads();
    // a run's start per creation arrival: the elements of buckets created later
    for (int k = t; k < nl; k += kUsT) W.mem[k] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kUsPer; ++j) {
      const int e = t + j * kUsT;
      if (e < nl && ct[j] == W.arr[e]) W.mem[ct[j]] = (int16_t)sz[j];
    }
    __syncthreads();
    {
      // suffix form: thread t over arrivals [nl - (t + 1) per, nl - t per), descending
      const int per = (nl + kUsT - 1) / kUsT;
      const int i1 = max(0, nl - t * per), i0 = max(0, i1 - per);
      int sum = 0;
      for (int k = i0; k < i1; ++k) sum += W.mem[k];
      int run;
      us_scan(sum, W.part, run);
      for (int k = i1 - 1; k >= i0; --k) {
        const int c = W.mem[k];
        W.mem[k] = (int16_t)run;
        run += c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kUsPer; ++j) {
      const int e = t + j * kUsT;
      if (e < nl) W.arr[e] = (int16_t)(W.mem[ct[j]] + rk[j]);
    }
    __syncthreads();
  }
  for (int e = t; e < n; e += kUsT) {
    const int o = W.arr[e];
    out[3 * o + 0] = pts[3 * e + 0];
    out[3 * o + 1] = pts[3 * e + 1];
    out[3 * o + 2] = pts[3 * e + 2];
  }
}

// the rehash points of a default-constructed std::unordered_map receiving
// n distinct keys one by one, from libstdc++'s own policy (max load 1, one
// bucket before the first insert): (elements before the insert, new count)
int umap_schedule(int64_t n, UmapSched* sc) {
  std::__detail::_Prime_rehash_policy pol;
  std::size_t nb = 1;
  sc->nl = 0;
  for (int64_t e = 0; e < n;) {
    const auto rh = pol._M_need_rehash(nb, (std::size_t)e, 1);
    if (rh.first) {
      if (sc->nl >= kUmapMaxLevels) return RST_E_ARG;
      sc->r[sc->nl] = e;
      sc->B[sc->nl] = (int64_t)rh.second;
      ++sc->nl;
      nb = rh.second;
    }
    // no rehash check fires before the element count passes _M_next_resize
    e = std::max<int64_t>(e + 1, std::min<int64_t>(n, (int64_t)pol._M_next_resize));
  }
  return RST_OK;
}

// out[0, n) = pts[0, n) (distinct voxels, insertion order) in the
// reference's unordered_map iteration order; kind / v as vox_coord
int umap_order_device(rst_ctx* ctx, const float* d_pts, int64_t n, float v, int kind, float* d_out) {
  if (n <= 0) return RST_OK;
  if (n >= ((int64_t)1 << 31) - 1) return RST_E_ARG;
  UmapSched sc;
  RST_CHECK(umap_schedule(n, &sc));
  const int64_t bmax = sc.B[sc.nl - 1];
  static const bool small_ok = [] {
    const char* e = getenv("RST_UMAP_SMALL");
    return !e || atoi(e) != 0;
  }();
  if (small_ok && n <= kUsMaxN && bmax <= kUsMaxB) {  // one CU, LDS (k_umap_small)
    k_umap_small<<<1, kUsT, 0, ctx->stream>>>(d_pts, (int)n, v, kind, sc, d_out);
    RST_HIP(hipGetLastError());
    return RST_OK;
  }
  const size_t bytes = sizeof(uint64_t) * n + sizeof(int32_t) * (6 * (size_t)n + 4 * (size_t)bmax) + 256;
  void* p = nullptr;
  size_t cls = 0;
  RST_CHECK(ctx_alloc(ctx, bytes, &p, &cls));
  UmapWs w;
  w.h = (uint64_t*)p;
  int32_t* q = (int32_t*)(w.h + n);
  w.pos = q;
  w.arr = q + n;
  w.bk = q + 2 * n;
  w.mem = q + 3 * n;
  w.hs = q + 4 * n;
  w.ctime = q + 6 * n;
  w.cnt = w.ctime + bmax;
  w.start = w.cnt + bmax;
  w.fill = w.start + bmax;
  k_umap_order<<<1, kUmapT, 0, ctx->stream>>>(d_pts, n, v, kind, sc, w, d_out);
  const hipError_t e = hipGetLastError();
  hipStreamSynchronize(ctx->stream);
  ctx_release(ctx, p, cls);
  RST_HIP(e);
  return RST_OK;
}

}  // namespace

int remove_nans_device(rst_ctx* ctx, const float* d_xyz, int64_t n, float* d_out,
                       int64_t* n_out) {
  if (n == 0) {
    *n_out = 0;
    return RST_OK;
  }
  const int nb = blocks_for(n, kTile);
  void* ws = nullptr;
  RST_CHECK(ctx_workspace(ctx, sizeof(uint32_t) * ((size_t)nb + 64), &ws));
  uint32_t* counts = (uint32_t*)ws;
  return compact(ctx, d_xyz, n, 0, nullptr, counts, counts + nb + 16, d_out, n_out);
}

// flag[i] = 1 iff point i is the first (lowest index) of its voxel; the
// workspace layout is returned so the caller can reuse its count buffer
struct VoxWs {
  uint8_t* flag;
  uint32_t* counts;
  int nb;
};

int first_per_voxel(rst_ctx* ctx, const float* d_xyz, int64_t n, float v, int kind,
                    VoxWs* out) {
  uint32_t slots = 1024;
  while ((int64_t)slots < 2 * n) slots <<= 1;
  const int nb = blocks_for(n, kTile);
  // workspace: rep[slots] | minidx[slots] | slot_of[n] | flag[n] | counts
  const size_t o_min = sizeof(int32_t) * slots;
  const size_t o_slot = o_min + sizeof(int32_t) * slots;
  const size_t o_flag = o_slot + sizeof(int32_t) * n;
  const size_t o_cnt = (o_flag + (size_t)n + 255) & ~(size_t)255;
  void* ws = nullptr;
  RST_CHECK(ctx_workspace(ctx, o_cnt + sizeof(uint32_t) * ((size_t)nb + 64), &ws));
  char* w = (char*)ws;
  int32_t* rep = (int32_t*)w;
  int32_t* minidx = (int32_t*)(w + o_min);
  int32_t* slot_of = (int32_t*)(w + o_slot);
  out->flag = (uint8_t*)(w + o_flag);
  out->counts = (uint32_t*)(w + o_cnt);
  out->nb = nb;
  hipStream_t st = ctx->stream;
  RST_HIP(hipMemsetAsync(rep, 0xff, sizeof(int32_t) * slots, st));     // -1: empty
  RST_HIP(hipMemsetAsync(minidx, 0x7f, sizeof(int32_t) * slots, st));  // > any index
  k_vox_claim<<<blocks_for(n), kBS, 0, st>>>(d_xyz, n, v, kind, rep, slots - 1, slot_of);
  k_vox_min<<<blocks_for(n), kBS, 0, st>>>(n, slot_of, minidx);
  k_vox_flag<<<blocks_for(n), kBS, 0, st>>>(n, slot_of, minidx, out->flag);
  RST_HIP(hipGetLastError());
  return RST_OK;
}

int downsample_voxel_device(rst_ctx* ctx, const float* d_xyz, int64_t n, float voxel,
                            float* d_out, int64_t* n_out) {
  if (n == 0) {
    *n_out = 0;
    return RST_OK;
  }
  VoxWs w;
  RST_CHECK(first_per_voxel(ctx, d_xyz, n, voxel, 0, &w));
  // the first point of each voxel in input order, then the reference's
  // unordered_map order (:54-57)
  float* tmp = nullptr;
  size_t cls = 0;
  RST_CHECK(ctx_alloc(ctx, sizeof(float) * 3 * (size_t)n, (void**)&tmp, &cls));
  int s = compact(ctx, d_xyz, n, 1, w.flag, w.counts, w.counts + w.nb + 16, tmp, n_out);
  if (s >= 0) s = umap_order_device(ctx, tmp, *n_out, voxel, 0, d_out);
  hipStreamSynchronize(ctx->stream);
  ctx_release(ctx, tmp, cls);
  return s;
}

// ---- CloudAccumulator (rs_replay_app.cpp:76-129) --------------------------------------
// A persistent voxel map: the first point ever added to each voxel, kept in
// insertion order.  Per AddCloud: transform (xfm * p, align_icp.cpp:107's
// order), the first point per voxel within the cloud (first_per_voxel,
// kind 1), then those representatives -- distinct keys -- are inserted into
// the persistent table (64-bit owner word per slot: cloud number << 32 |
// index; a slot owned by the current cloud holds a different key, one owned
// by an earlier cloud has its key visible and is compared), and the inserted
// ones are appended to the point list with an order-preserving compaction.
// The table is rebuilt from the list when it passes half full.
constexpr uint64_t kAccEmpty = ~0ull;
constexpr uint32_t kAccRebuilt = 0xFFFFFFFEu;

__global__ __launch_bounds__(kBS) void k_acc_xform(const float* __restrict__ xyz, int64_t n,
                                                   Pose3 P, float* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  float x, y, z;
  xform(P, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], x, y, z);
  out[3 * i] = x;
  out[3 * i + 1] = y;
  out[3 * i + 2] = z;
}

__global__ __launch_bounds__(kBS) void k_acc_insert(const float* __restrict__ xyz, int64_t n,
                                                    const uint8_t* __restrict__ first, float inv,
                                                    uint64_t* __restrict__ owner,
                                                    int32_t* __restrict__ keys, uint32_t mask,
                                                    uint32_t cloud, uint8_t* __restrict__ ins) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  if (!first[i]) {
    ins[i] = 0;
    return;
  }
  const Vox k = vox_of(xyz, i, inv, 1);
  const uint64_t mine = ((uint64_t)cloud << 32) | (uint64_t)(uint32_t)i;
  uint32_t h = vox_hash(k) & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    uint64_t o = __hip_atomic_load(&owner[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (o == kAccEmpty) {
      const uint64_t prev = atomicCAS((unsigned long long*)&owner[h], kAccEmpty, mine);
      if (prev == kAccEmpty) {
        keys[3 * h] = k.x;
        keys[3 * h + 1] = k.y;
        keys[3 * h + 2] = k.z;
        ins[i] = 1;
        return;
      }
      o = prev;
    }
    // a slot taken in this launch holds another key (the representatives'
    // keys are distinct); earlier slots' keys are visible: compare
    if ((uint32_t)(o >> 32) != cloud && keys[3 * h] == k.x && keys[3 * h + 1] == k.y &&
        keys[3 * h + 2] == k.z) {
      ins[i] = 0;  // the voxel already has its point (emplace only when new)
      return;
    }
    h = (h + 1) & mask;
  }
  ins[i] = 0;  // unreachable: the table stays at most half full
}

// re-insert every list point (distinct keys by construction)
__global__ __launch_bounds__(kBS) void k_acc_rebuild(const float* __restrict__ list, int64_t n,
                                                     float inv, uint64_t* __restrict__ owner,
                                                     int32_t* __restrict__ keys, uint32_t mask) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  const Vox k = vox_of(list, i, inv, 1);
  const uint64_t mine = ((uint64_t)kAccRebuilt << 32) | (uint64_t)(uint32_t)i;
  uint32_t h = vox_hash(k) & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    if (atomicCAS((unsigned long long*)&owner[h], kAccEmpty, mine) == kAccEmpty) {
      keys[3 * h] = k.x;
      keys[3 * h + 1] = k.y;
      keys[3 * h + 2] = k.z;
      return;
    }
    h = (h + 1) & mask;
  }
}

}  // namespace rst

using namespace rst;

namespace {

// host-buffer entry points: upload, run `fn` on device buffers, download --
// both copies through the context's pinned staging buffer (stage_h2d /
// stage_d2h: bounded chunks, as capi.hip's uploads).  A copy straight from / to pageable memory leaves the pinning to
// the runtime, which measured 20-28 ms on a frame not copied recently
// (profiles/r05_callers_prof.txt: the first RemoveNans of each pair of the
// callers' workload, 0.4 ms otherwise); a staged copy is a host memcpy plus
// a pinned DMA every time.
template <class Fn>
int run_host(rst_ctx* ctx, const float* xyz, int64_t n, float* out, int64_t* n_out, Fn fn) {
  float *din = nullptr, *dout = nullptr;
  size_t cin = 0, cout = 0;
  const size_t bytes = sizeof(float) * 3 * (size_t)std::max<int64_t>(n, 1);
  RST_CHECK(ctx_alloc(ctx, bytes, (void**)&din, &cin));
  int s = ctx_alloc(ctx, bytes, (void**)&dout, &cout);
  if (s >= 0 && n > 0) s = stage_h2d(ctx, din, xyz, sizeof(float) * 3 * n);
  if (s >= 0) s = fn(din, dout);
  if (s >= 0 && *n_out > 0) s = stage_d2h(ctx, out, dout, sizeof(float) * 3 * (*n_out));
  hipStreamSynchronize(ctx->stream);
  ctx_release(ctx, din, cin);
  if (dout) ctx_release(ctx, dout, cout);
  return s < 0 ? s : RST_OK;
}

}  // namespace

extern "C" {

int rst_remove_nans_device(rst_ctx* ctx, const float* d_xyz, int64_t n, float* d_out,
                           int64_t* n_out) {
  if (!ctx || n < 0 || !n_out || (n > 0 && (!d_xyz || !d_out))) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return remove_nans_device(ctx, d_xyz, n, d_out, n_out);
}

int rst_remove_nans(rst_ctx* ctx, const float* xyz, int64_t n, float* out, int64_t* n_out) {
  if (!ctx || n < 0 || !n_out || (n > 0 && (!xyz || !out))) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  *n_out = 0;
  return run_host(ctx, xyz, n, out, n_out, [&](const float* din, float* dout) {
    return remove_nans_device(ctx, din, n, dout, n_out);
  });
}

int rst_downsample_voxel_device(rst_ctx* ctx, const float* d_xyz, int64_t n, float voxel_size,
                                float* d_out, int64_t* n_out) {
  if (!ctx || n < 0 || !n_out || (n > 0 && (!d_xyz || !d_out)) || !(voxel_size > 0.f))
    return RST_E_ARG;
  if (n >= ((int64_t)1 << 30)) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return downsample_voxel_device(ctx, d_xyz, n, voxel_size, d_out, n_out);
}

int rst_downsample_voxel(rst_ctx* ctx, const float* xyz, int64_t n, float voxel_size, float* out,
                         int64_t* n_out) {
  if (!ctx || n < 0 || !n_out || (n > 0 && (!xyz || !out)) || !(voxel_size > 0.f))
    return RST_E_ARG;
  if (n >= ((int64_t)1 << 30)) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  *n_out = 0;
  return run_host(ctx, xyz, n, out, n_out, [&](const float* din, float* dout) {
    return downsample_voxel_device(ctx, din, n, voxel_size, dout, n_out);
  });
}

}  // extern "C"

// ---- CloudAccumulator handle ----------------------------------------------------------
struct rst_accum {
  rst_ctx* ctx = nullptr;
  float voxel = 0.f, inv = 0.f;
  uint32_t cap = 0;        // table slots (power of two)
  uint64_t* owner = nullptr;
  int32_t* keys = nullptr;  // 3 per slot
  float* list = nullptr;    // accumulated points, insertion order
  int64_t count = 0, list_cap = 0;
  uint32_t cloud = 0;       // AddCloud calls so far
};

namespace {

int accum_grow_table(rst_accum* a, int64_t need) {
  uint32_t cap = a->cap ? a->cap : 1u << 16;
  while ((int64_t)cap < 2 * need) cap <<= 1;
  if (cap == a->cap && a->owner) return RST_OK;
  hipStream_t st = a->ctx->stream;
  RST_HIP(hipStreamSynchronize(st));
  if (a->owner) hipFree(a->owner);
  if (a->keys) hipFree(a->keys);
  a->owner = nullptr;
  a->keys = nullptr;
  if (hipMalloc(&a->owner, sizeof(uint64_t) * cap) != hipSuccess ||
      hipMalloc(&a->keys, sizeof(int32_t) * 3 * cap) != hipSuccess)
    return RST_E_NOMEM;
  a->cap = cap;
  RST_HIP(hipMemsetAsync(a->owner, 0xff, sizeof(uint64_t) * cap, st));
  if (a->count > 0) {
    k_acc_rebuild<<<(unsigned)((a->count + kBS - 1) / kBS), kBS, 0, st>>>(
        a->list, a->count, a->inv, a->owner, a->keys, cap - 1);
    RST_HIP(hipGetLastError());
  }
  return RST_OK;
}

int accum_grow_list(rst_accum* a, int64_t need) {
  if (need <= a->list_cap) return RST_OK;
  int64_t cap = a->list_cap ? a->list_cap : 1 << 16;
  while (cap < need) cap *= 2;
  float* nl = nullptr;
  if (hipMalloc(&nl, sizeof(float) * 3 * cap) != hipSuccess) return RST_E_NOMEM;
  if (a->count > 0)
    RST_HIP(hipMemcpyAsync(nl, a->list, sizeof(float) * 3 * a->count, hipMemcpyDeviceToDevice,
                           a->ctx->stream));
  RST_HIP(hipStreamSynchronize(a->ctx->stream));
  if (a->list) hipFree(a->list);
  a->list = nl;
  a->list_cap = cap;
  return RST_OK;
}

int accum_add_device(rst_accum* a, const float pose[16], const float* d_xyz, int64_t n) {
  if (n == 0) return RST_OK;
  rst_ctx* ctx = a->ctx;
  hipStream_t st = ctx->stream;
  RST_CHECK(accum_grow_table(a, a->count + n));
  RST_CHECK(accum_grow_list(a, a->count + n));
  float* tmp = nullptr;
  uint8_t* ins = nullptr;
  size_t ct = 0, ci = 0;
  RST_CHECK(ctx_alloc(ctx, sizeof(float) * 3 * n, (void**)&tmp, &ct));
  int s = ctx_alloc(ctx, (size_t)n, (void**)&ins, &ci);
  if (s >= 0) {
    Pose3 P;
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) P.r[3 * c + r] = pose[4 * c + r];  // column-major
    for (int r = 0; r < 3; ++r) P.t[r] = pose[12 + r];
    k_acc_xform<<<blocks_for(n), kBS, 0, st>>>(d_xyz, n, P, tmp);
    VoxWs w;
    s = first_per_voxel(ctx, tmp, n, a->inv, 1, &w);
    if (s >= 0) {
      k_acc_insert<<<blocks_for(n), kBS, 0, st>>>(tmp, n, w.flag, a->inv, a->owner, a->keys,
                                                  a->cap - 1, a->cloud, ins);
      int64_t added = 0;
      s = compact(ctx, tmp, n, 1, ins, w.counts, w.counts + w.nb + 16, a->list + 3 * a->count,
                  &added);
      if (s >= 0) {
        a->count += added;
        a->cloud = a->cloud + 1 >= kAccRebuilt ? 0 : a->cloud + 1;
      }
    }
  }
  hipStreamSynchronize(st);
  ctx_release(ctx, tmp, ct);
  if (ins) ctx_release(ctx, ins, ci);
  return s < 0 ? s : RST_OK;
}

}  // namespace

extern "C" {

int rst_accum_create(rst_ctx* ctx, float voxel_size, rst_accum** out) {
  if (!ctx || !out || !(voxel_size > 0.f)) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  rst_accum* a = new rst_accum();
  a->ctx = ctx;
  a->voxel = voxel_size;
  a->inv = (float)(1.0 / (double)voxel_size);  // voxel_size_inv_(1.0 / voxel_size_)
  *out = a;
  return RST_OK;
}

int rst_accum_destroy(rst_accum* a) {
  if (!a) return RST_OK;
  if (a->ctx) hipStreamSynchronize(a->ctx->stream);
  if (a->owner) hipFree(a->owner);
  if (a->keys) hipFree(a->keys);
  if (a->list) hipFree(a->list);
  delete a;
  return RST_OK;
}

int rst_accum_add_device(rst_accum* a, const float pose[16], const float* d_xyz, int64_t n) {
  if (!a || !pose || n < 0 || (n > 0 && !d_xyz) || n >= ((int64_t)1 << 30)) return RST_E_ARG;
  RST_HIP(hipSetDevice(a->ctx->device));
  return accum_add_device(a, pose, d_xyz, n);
}

int rst_accum_add(rst_accum* a, const float pose[16], const float* xyz, int64_t n) {
  if (!a || !pose || n < 0 || (n > 0 && !xyz) || n >= ((int64_t)1 << 30)) return RST_E_ARG;
  RST_HIP(hipSetDevice(a->ctx->device));
  if (n == 0) return RST_OK;
  float* d = nullptr;
  size_t c = 0;
  RST_CHECK(ctx_alloc(a->ctx, sizeof(float) * 3 * n, (void**)&d, &c));
  // staged through pinned memory (run_host above: no pageable-copy stall)
  int s = stage_h2d(a->ctx, d, xyz, sizeof(float) * 3 * n);
  if (s >= 0) s = accum_add_device(a, pose, d, n);
  hipStreamSynchronize(a->ctx->stream);
  ctx_release(a->ctx, d, c);
  return s;
}

int rst_accum_size(const rst_accum* a, int64_t* n) {
  if (!a || !n) return RST_E_ARG;
  *n = a->count;
  return RST_OK;
}

int rst_accum_extract(rst_accum* a, float* out, int64_t* n_out) {
  if (!a || !n_out || (a->count > 0 && !out)) return RST_E_ARG;
  RST_HIP(hipSetDevice(a->ctx->device));
  if (a->count > 0) {
    // the insertion-ordered list in the reference's unordered_map order
    // (rs_replay_app.cpp:112-121), then to the host
    float* tmp = nullptr;
    size_t cls = 0;
    RST_CHECK(ctx_alloc(a->ctx, sizeof(float) * 3 * (size_t)a->count, (void**)&tmp, &cls));
    int s = umap_order_device(a->ctx, a->list, a->count, a->inv, 1, tmp);
    if (s >= 0) s = stage_d2h(a->ctx, out, tmp, sizeof(float) * 3 * a->count);
    hipStreamSynchronize(a->ctx->stream);
    ctx_release(a->ctx, tmp, cls);
    RST_CHECK(s);
  }
  *n_out = a->count;
  return RST_OK;
}

}  // extern "C"

extern "C" int rst_debug_umap_schedule(int64_t n, int64_t* out, int64_t cap, int64_t* count) {
  if (n < 0 || !count || (cap > 0 && !out)) return RST_E_ARG;
  rst::UmapSched sc;
  RST_CHECK(rst::umap_schedule(n, &sc));
  for (int k = 0; k < sc.nl && k < cap; ++k) {
    out[2 * k] = sc.r[k];
    out[2 * k + 1] = sc.B[k];
  }
  *count = sc.nl;
  return RST_OK;
}
