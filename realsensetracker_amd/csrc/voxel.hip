// voxel.hip -- the preprocessing every reference caller runs right before
// AlignIcp3d (rs_replay_app.cpp:229,246-247,
// rs_align_app.cpp:254-255):
//
//   RemoveNans      (point_cloud_utils.cpp:163-174): drop points with a
//                   non-finite coordinate, order kept;
//   DownsampleVoxel (point_cloud_utils.cpp:34-68): one point per voxel
//                   floor(p / voxel_size) -- the FIRST point (lowest index)
//                   of each voxel, since the reference emplaces only when the
//                   key is new.  The reference emits them in unordered_map
//                   order (implementation-defined); here they come out in
//                   ascending input index (deterministic).  The voxel key is
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

// (int)floor(x / v) with x86-64 cvttss2si semantics outside int range / NaN
__device__ __forceinline__ int vox_coord(float x, float v) {
  const float q = floorf(x / v);
  return (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT_MIN;
}

struct Vox {
  int x, y, z;
};

__device__ __forceinline__ Vox vox_of(const float* __restrict__ xyz, int64_t i, float v) {
  return Vox{vox_coord(xyz[3 * i], v), vox_coord(xyz[3 * i + 1], v),
             vox_coord(xyz[3 * i + 2], v)};
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
                                                   float v, int32_t* __restrict__ rep,
                                                   uint32_t mask, int32_t* __restrict__ slot_of) {
  const int64_t i = blockIdx.x * (int64_t)kBS + threadIdx.x;
  if (i >= n) return;
  const Vox k = vox_of(xyz, i, v);
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
    const Vox o = vox_of(xyz, cur, v);
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

int downsample_voxel_device(rst_ctx* ctx, const float* d_xyz, int64_t n, float voxel,
                            float* d_out, int64_t* n_out) {
  if (n == 0) {
    *n_out = 0;
    return RST_OK;
  }
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
  uint8_t* flag = (uint8_t*)(w + o_flag);
  uint32_t* counts = (uint32_t*)(w + o_cnt);
  hipStream_t st = ctx->stream;
  RST_HIP(hipMemsetAsync(rep, 0xff, sizeof(int32_t) * slots, st));     // -1: empty
  RST_HIP(hipMemsetAsync(minidx, 0x7f, sizeof(int32_t) * slots, st));  // > any index
  k_vox_claim<<<blocks_for(n), kBS, 0, st>>>(d_xyz, n, voxel, rep, slots - 1, slot_of);
  k_vox_min<<<blocks_for(n), kBS, 0, st>>>(n, slot_of, minidx);
  k_vox_flag<<<blocks_for(n), kBS, 0, st>>>(n, slot_of, minidx, flag);
  RST_HIP(hipGetLastError());
  return compact(ctx, d_xyz, n, 1, flag, counts, counts + nb + 16, d_out, n_out);
}

}  // namespace rst

using namespace rst;

namespace {

// host-buffer entry points: upload, run `fn` on device buffers, download
template <class Fn>
int run_host(rst_ctx* ctx, const float* xyz, int64_t n, float* out, int64_t* n_out, Fn fn) {
  float *din = nullptr, *dout = nullptr;
  size_t cin = 0, cout = 0;
  const size_t bytes = sizeof(float) * 3 * (size_t)std::max<int64_t>(n, 1);
  RST_CHECK(ctx_alloc(ctx, bytes, (void**)&din, &cin));
  int s = ctx_alloc(ctx, bytes, (void**)&dout, &cout);
  if (s >= 0 && n > 0 &&
      hipMemcpyAsync(din, xyz, sizeof(float) * 3 * n, hipMemcpyHostToDevice, ctx->stream) !=
          hipSuccess)
    s = RST_E_HIP;
  if (s >= 0) s = fn(din, dout);
  if (s >= 0 && *n_out > 0 &&
      (hipMemcpyAsync(out, dout, sizeof(float) * 3 * (*n_out), hipMemcpyDeviceToHost,
                      ctx->stream) != hipSuccess ||
       hipStreamSynchronize(ctx->stream) != hipSuccess))
    s = RST_E_HIP;
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
