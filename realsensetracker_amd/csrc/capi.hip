// capi.hip -- extern "C" entry points of include/rst_align.h.
//
// Host-pointer entry points stage through the context's pinned buffer and
// device workspace; *_device entry points take HBM pointers directly.
#include <hip/hip_runtime.h>

#include <chrono>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "rst_internal.hpp"

namespace rst {

static thread_local char g_last_error[512] = {0};

// Kernel arguments in device memory unless the environment says otherwise:
// with the runtime's default (host memory) every kernel's first argument
// load waited ~6k clocks on the host link (measured in k_sq_walk: its
// prologue 7.7k -> 1.5k clocks).  Read by the HIP runtime when it
// initialises, so set at load time, before this library's first HIP call.
// The variable is process-wide: it also places the kernel arguments of any
// other HIP code in the process that initialises the runtime afterwards
// (INTEGRATION.md).  A set value is never overridden, and
// RST_NO_ENV_DEFAULTS=1 leaves the environment untouched (the loader sets
// nothing either; a host that initialises HIP before loading this library
// keeps its own placement).
__attribute__((constructor)) static void rst_env_defaults() {
  const char* off = getenv("RST_NO_ENV_DEFAULTS");
  if (off && *off && *off != '0') return;
  setenv("HIP_FORCE_DEV_KERNARG", "1", 0);
}

void set_last_error(hipError_t e, const char* what, const char* file, int line) {
  snprintf(g_last_error, sizeof(g_last_error), "%s failed: %s (%s:%d)", what,
           hipGetErrorString(e), file, line);
  if (getenv("RST_VERBOSE")) fprintf(stderr, "[rst] %s\n", g_last_error);
}

static size_t size_class(size_t bytes) {
  size_t b = bytes < 256 ? 256 : bytes;
  int lg = 63 - __builtin_clzll(b);
  const size_t step = lg >= 3 ? ((size_t)1 << (lg - 3)) : 1;
  return (b + step - 1) / step * step;
}

constexpr size_t kPoolMaxBytes = (size_t)4 << 30;

int ctx_alloc(rst_ctx* ctx, size_t bytes, void** out, size_t* class_bytes) {
  const size_t c = size_class(bytes);
  *class_bytes = c;
  std::lock_guard<std::mutex> lk(ctx->pool_mu);
  auto it = ctx->pool.find(c);
  if (it != ctx->pool.end()) {
    *out = it->second;
    ctx->pool.erase(it);
    ctx->pool_bytes -= c;
    return RST_OK;
  }
  if (hipMalloc(out, c) != hipSuccess) {
    // give the cached blocks back and retry once
    for (auto& kv : ctx->pool) hipFree(kv.second);
    ctx->pool.clear();
    ctx->pool_bytes = 0;
    if (hipMalloc(out, c) != hipSuccess) return RST_E_NOMEM;
  }
  return RST_OK;
}

void ctx_release(rst_ctx* ctx, void* p, size_t c) {
  if (!p) return;
  if (ctx) {
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    if (ctx->pool_bytes + c <= kPoolMaxBytes) {
      ctx->pool.emplace(c, p);
      ctx->pool_bytes += c;
      return;
    }
  }
  hipFree(p);
}

int target_alloc(rst_target* t, size_t bytes, void** out) {
  size_t c = 0;
  RST_CHECK(ctx_alloc(t->ctx, bytes, out, &c));
  t->allocs.emplace_back(*out, c);
  return RST_OK;
}

int ctx_workspace(rst_ctx* ctx, size_t bytes, void** out) {
  if (bytes > ctx->ws_bytes) {
    if (ctx->ws) {
      RST_HIP(hipStreamSynchronize(ctx->stream));
      RST_HIP(hipFree(ctx->ws));
      ctx->ws = nullptr;
      ctx->ws_bytes = 0;
    }
    const size_t sz = std::max<size_t>(bytes + bytes / 4, 1 << 20);
    if (hipMalloc(&ctx->ws, sz) != hipSuccess) return RST_E_NOMEM;
    ctx->ws_bytes = sz;
  }
  *out = ctx->ws;
  return RST_OK;
}

static int stage_init(rst_ctx* ctx) {
  if (ctx->pinned) return RST_OK;
  const size_t sz = 2 * kStageChunk + kPinnedSmall;
  if (hipHostMalloc(&ctx->pinned, sz, hipHostMallocDefault) != hipSuccess) return RST_E_NOMEM;
  ctx->pinned_bytes = sz;
  for (int k = 0; k < 2; ++k) {
    RST_HIP(hipEventCreateWithFlags(&ctx->stage_ev[k], hipEventDisableTiming));
    RST_HIP(hipEventRecord(ctx->stage_ev[k], ctx->stream));
  }
  return RST_OK;
}

int ctx_pinned_small(rst_ctx* ctx, size_t bytes, void** out) {
  if (bytes > kPinnedSmall) return RST_E_ARG;
  RST_CHECK(stage_init(ctx));
  *out = (char*)ctx->pinned + 2 * kStageChunk;
  return RST_OK;
}

int stage_h2d(rst_ctx* ctx, void* d, const void* h, size_t bytes) {
  if (bytes == 0) return RST_OK;
  RST_CHECK(stage_init(ctx));
  for (size_t off = 0, i = 0; off < bytes; off += kStageChunk, ++i) {
    const int k = (int)(i & 1);
    const size_t len = std::min(kStageChunk, bytes - off);
    char* pin = (char*)ctx->pinned + k * kStageChunk;
    RST_HIP(hipEventSynchronize(ctx->stage_ev[k]));  // the half's previous DMA is done
    memcpy(pin, (const char*)h + off, len);
    RST_HIP(hipMemcpyAsync((char*)d + off, pin, len, hipMemcpyHostToDevice, ctx->stream));
    RST_HIP(hipEventRecord(ctx->stage_ev[k], ctx->stream));
  }
  return RST_OK;
}

int stage_d2h(rst_ctx* ctx, void* h, const void* d, size_t bytes) {
  if (bytes == 0) return RST_OK;
  RST_CHECK(stage_init(ctx));
  const size_t nc = (bytes + kStageChunk - 1) / kStageChunk;
  auto issue = [&](size_t i) -> int {
    const int k = (int)(i & 1);
    const size_t off = i * kStageChunk, len = std::min(kStageChunk, bytes - off);
    RST_HIP(hipEventSynchronize(ctx->stage_ev[k]));
    RST_HIP(hipMemcpyAsync((char*)ctx->pinned + k * kStageChunk, (const char*)d + off, len,
                           hipMemcpyDeviceToHost, ctx->stream));
    RST_HIP(hipEventRecord(ctx->stage_ev[k], ctx->stream));
    return RST_OK;
  };
  RST_CHECK(issue(0));
  for (size_t i = 0; i < nc; ++i) {
    const int k = (int)(i & 1);
    const size_t off = i * kStageChunk, len = std::min(kStageChunk, bytes - off);
    if (i + 1 < nc) RST_CHECK(issue(i + 1));  // (the other half: in flight meanwhile)
    RST_HIP(hipEventSynchronize(ctx->stage_ev[k]));
    memcpy((char*)h + off, (const char*)ctx->pinned + k * kStageChunk, len);
  }
  return RST_OK;
}

int ctx_slab(rst_ctx* ctx, size_t bytes, double** out) {
  if (bytes > ctx->slab_bytes) {
    if (ctx->d_slab) {
      RST_HIP(hipStreamSynchronize(ctx->stream));
      RST_HIP(hipFree(ctx->d_slab));
      ctx->d_slab = nullptr;
      ctx->slab_bytes = 0;
    }
    const size_t sz = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    if (hipMalloc(&ctx->d_slab, sz) != hipSuccess) return RST_E_NOMEM;
    ctx->slab_bytes = sz;
  }
  *out = ctx->d_slab;
  return RST_OK;
}

// Upload host AoS xyz (n points) into a device buffer from the context's
// size-class pool (no hipMalloc / hipFree per call: hipFree synchronises the
// whole device); give it back with free_xyz.
static size_t xyz_bytes(int64_t n) { return sizeof(float) * 3 * (size_t)std::max<int64_t>(n, 1); }

static void free_xyz(rst_ctx* ctx, float* d, int64_t n) {
  if (!d) return;
  (void)hipStreamSynchronize(ctx->stream);  // no kernel may still read it
  ctx_release(ctx, d, size_class(xyz_bytes(n)));
}

static int upload_xyz(rst_ctx* ctx, const float* h, int64_t n, float** d_out) {
  *d_out = nullptr;
  const size_t bytes = xyz_bytes(n);
  void* dv = nullptr;
  size_t cls = 0;
  RST_CHECK(ctx_alloc(ctx, bytes, &dv, &cls));
  float* d = (float*)dv;
  if (n > 0) {
    const int s = stage_h2d(ctx, d, h, sizeof(float) * 3 * n);
    if (s < 0) {
      free_xyz(ctx, d, n);
      return s;
    }
  }
  *d_out = d;
  return RST_OK;
}

// the measured HBM ceiling (rst_debug_stream_copy): a float4 copy, U float4
// per thread in flight (all loads before the stores), nontemporal or default
// cache policy; the best of the variants is the ceiling
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_stream_copy(const float4* __restrict__ a,
                                                     float4* __restrict__ b, int64_t n4) {
  const f32x4* __restrict__ av = reinterpret_cast<const f32x4*>(a);
  f32x4* __restrict__ bv = reinterpret_cast<f32x4*>(b);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; i0 < n4; i0 += stride) {
    f32x4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < n4) t[u] = NT ? __builtin_nontemporal_load(av + i) : av[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * blockDim.x;
      if (i < n4) {
        if (NT)
          __builtin_nontemporal_store(t[u], bv + i);
        else
          bv[i] = t[u];
      }
    }
  }
}

// the dispatch-rate probe (rst_debug_launch_rate): a kernel that does
// nothing but exist (one vector store per block to lane 0's slot)
__global__ void k_nop(int* __restrict__ sink, int tag) {
  if (threadIdx.x == 0 && tag < 0) sink[blockIdx.x] = tag;
}

// the concurrency probe (rst_debug_kernel_overlap): every wave waits
// `ticks` of the 100 MHz real-time clock (no memory traffic, no ALU
// pressure), holding `lds` bytes of dynamic LDS -- how many such kernels
// from independent streams the GPU runs at once
__global__ void k_spin(int* __restrict__ sink, int tag, int ticks) {
  extern __shared__ int spin_lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0 && tag < 0) sink[blockIdx.x] = tag + spin_lds[0];
}

}  // namespace rst

using namespace rst;

#include "rst_debug.h"

extern "C" {

int rst_abi_version(void) { return RST_ABI_VERSION; }

const char* rst_status_string(int s) {
  switch (s) {
    case RST_OK: return "ok";
    case RST_FALSE: return "false (reference failure condition)";
    case RST_E_ARG: return "invalid argument";
    case RST_E_HIP: return g_last_error[0] ? g_last_error : "HIP error";
    case RST_E_NOMEM: return "out of memory";
    case RST_E_NODEVICE: return "no GPU device";
    case RST_E_COMM: return "RCCL error";
    case RST_E_STATE: return "object in wrong state";
    default: return "unknown status";
  }
}

void rst_icp_opts_default(rst_icp_opts* o) {
  if (!o) return;
  memset(o, 0, sizeof(*o));
  o->max_iter = 128;         // rs_align_app.cpp:303, rs_replay_app.cpp:251
  o->mode = RST_P2POINT_REF;
  o->mu0 = 1.0f;             // align_icp.cpp:91
  o->anneal_every = 8;       // :96
  o->anneal_div = 1.4f;      // :97
  o->p2plane_eps = 1e-6f;
  o->p2plane_mu = 4e-4f;     // (2 cm)^2
  o->p2plane_max_dist = 0.0f;
}

int rst_device_count(int* count) {
  if (!count) return RST_E_ARG;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *count = c;
  return RST_OK;
}

int rst_ctx_create(int device, rst_ctx** out) {
  if (!out) return RST_E_ARG;
  *out = nullptr;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || c <= 0) return RST_E_NODEVICE;
  if (device < 0 || device >= c) return RST_E_NODEVICE;
  RST_HIP(hipSetDevice(device));
  rst_ctx* ctx = new rst_ctx();
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&ctx->d_state, sizeof(IcpState)) != hipSuccess ||
      hipHostMalloc(&ctx->h_state, sizeof(IcpState), hipHostMallocDefault) != hipSuccess) {
    rst_ctx_destroy(ctx);
    return RST_E_HIP;
  }
  ctx->stream = ctx->own_stream;
  *out = ctx;
  return RST_OK;
}

int rst_ctx_destroy(rst_ctx* ctx) {
  if (!ctx) return RST_OK;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  for (hipEvent_t e : ctx->ev) hipEventDestroy(e);
  for (auto& kv : ctx->gexec) hipGraphExecDestroy(kv.second);
  if (ctx->ws) hipFree(ctx->ws);
  if (ctx->pinned) hipHostFree(ctx->pinned);
  for (hipEvent_t e : ctx->stage_ev)
    if (e) hipEventDestroy(e);
  if (ctx->d_state) hipFree(ctx->d_state);
  if (ctx->h_state) hipHostFree(ctx->h_state);
  if (ctx->d_bstate) hipFree(ctx->d_bstate);
  if (ctx->h_bstate) hipHostFree(ctx->h_bstate);
  if (ctx->d_slab) hipFree(ctx->d_slab);
  if (ctx->d_sqstats) hipFree(ctx->d_sqstats);
  if (ctx->own_stream) hipStreamDestroy(ctx->own_stream);
  for (rst_target* t : ctx->live) t->ctx = nullptr;  // they free to the device
  for (auto& kv : ctx->pool) hipFree(kv.second);
  delete ctx;
  return RST_OK;
}

int rst_ctx_set_stream(rst_ctx* ctx, void* s) {
  if (!ctx) return RST_E_ARG;
  ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
  return RST_OK;
}

int rst_ctx_synchronize(rst_ctx* ctx) {
  if (!ctx) return RST_E_ARG;
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return RST_OK;
}

int rst_ctx_last_kernel_time(rst_ctx* ctx, float* avg_ms, int32_t* launches) {
  if (!ctx) return RST_E_ARG;
  if (avg_ms) *avg_ms = ctx->last_kernel_ms;
  if (launches) *launches = ctx->last_kernel_launches;
  return RST_OK;
}

int rst_ctx_last_iteration_times(rst_ctx* ctx, float avg_ms[3], int32_t* iterations) {
  if (!ctx || !avg_ms) return RST_E_ARG;
  for (int k = 0; k < 3; ++k) avg_ms[k] = ctx->last_iter_ms[k];
  if (iterations) *iterations = ctx->last_kernel_launches;
  return RST_OK;
}

int rst_ctx_last_iterations(rst_ctx* ctx, int32_t* iterations) {
  if (!ctx || !iterations) return RST_E_ARG;
  *iterations = ctx->last_iters;
  return RST_OK;
}

int rst_ctx_enable_graphs(rst_ctx* ctx, int enable) {
  if (!ctx) return RST_E_ARG;
  ctx->graphs = enable != 0;
  return RST_OK;
}

int rst_debug_enable_seq_trace(rst_ctx* ctx, int enable) {
  if (!ctx) return RST_E_ARG;
  ctx->seq_trace = enable != 0;
  if (ctx->seq_trace && !ctx->d_sqstats) {
    RST_HIP(hipSetDevice(ctx->device));
    if (hipMalloc(&ctx->d_sqstats, sizeof(int32_t) * 64 * kQTrace) != hipSuccess) return RST_E_NOMEM;
    RST_HIP(hipMemset(ctx->d_sqstats, 0, sizeof(int32_t) * 64 * kQTrace));
  }
  return RST_OK;
}

int rst_debug_seqsum_fault(rst_ctx* ctx, int32_t bits) {
  if (!ctx || bits < 0 || bits > 127) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return seqsum_debug_fault((int)bits);
}

int rst_debug_wave_scan(rst_ctx* ctx, const double* in, double* out) {
  if (!ctx || !in || !out) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return seqsum_debug_wave_scan(ctx->stream, in, out);
}

int rst_debug_seq_walk_stats(rst_ctx* ctx, int32_t* out, int32_t n) {
  if (!ctx || !out || n < 0 || !ctx->d_sqstats) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  RST_HIP(hipMemcpy(out, ctx->d_sqstats, sizeof(int32_t) * 64 * std::min<int32_t>(n, kQTrace),
                    hipMemcpyDeviceToHost));
  return RST_OK;
}

int rst_debug_seq_trace(rst_ctx* ctx, float* out, int32_t n) {
  if (!ctx || !out || n < 0) return RST_E_ARG;
  for (int i = 0; i < n && i < kQTrace; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = ctx->h_state->seqtr[i][j];
  return RST_OK;
}

// the last batch's pair `pair` (its index in the call): its per-iteration
// sequential sums (rst_debug_seq_trace's layout; the batched loop walks the
// cost chain in the last iteration only, so column 3 is valid there alone)
int rst_debug_batch_seq_trace(rst_ctx* ctx, int32_t pair, float* out, int32_t n) {
  if (!ctx || !out || n < 0 || pair < 0 || pair >= ctx->bpend.nb || ctx->bpend.active) return RST_E_ARG;
  const int slot = ctx->bpend.slot[pair];
  if (slot < 0 || !ctx->h_bstate) return RST_E_STATE;
  for (int i = 0; i < n && i < kQTrace; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = ctx->h_bstate[slot].seqtr[i][j];
  return RST_OK;
}

int rst_ctx_enable_kernel_timing(rst_ctx* ctx, int enable) {
  if (!ctx) return RST_E_ARG;
  ctx->timing = enable != 0;
  ctx->timing_stride = enable > 1 ? enable : 1;
  return RST_OK;
}

// ---- device buffers ------------------------------------------------------------
int rst_dev_alloc(rst_ctx* ctx, int64_t bytes, void** d_out) {
  if (!ctx || !d_out || bytes < 0) return RST_E_ARG;
  *d_out = nullptr;
  RST_HIP(hipSetDevice(ctx->device));
  if (hipMalloc(d_out, (size_t)std::max<int64_t>(bytes, 1)) != hipSuccess) return RST_E_NOMEM;
  return RST_OK;
}

int rst_dev_free(rst_ctx* ctx, void* d) {
  if (!ctx) return RST_E_ARG;
  if (!d) return RST_OK;
  RST_HIP(hipSetDevice(ctx->device));
  RST_HIP(hipStreamSynchronize(ctx->stream));  // no pending work may still use it
  RST_HIP(hipFree(d));
  return RST_OK;
}

int rst_dev_upload(rst_ctx* ctx, void* d_dst, const void* h_src, int64_t bytes) {
  if (!ctx || bytes < 0 || (bytes > 0 && (!d_dst || !h_src))) return RST_E_ARG;
  if (bytes == 0) return RST_OK;
  RST_HIP(hipSetDevice(ctx->device));
  RST_HIP(hipMemcpyAsync(d_dst, h_src, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return RST_OK;
}

int rst_dev_download(rst_ctx* ctx, void* h_dst, const void* d_src, int64_t bytes) {
  if (!ctx || bytes < 0 || (bytes > 0 && (!d_src || !h_dst))) return RST_E_ARG;
  if (bytes == 0) return RST_OK;
  RST_HIP(hipSetDevice(ctx->device));
  RST_HIP(hipMemcpyAsync(h_dst, d_src, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return RST_OK;
}

// ---- target ------------------------------------------------------------------
int rst_target_build(rst_ctx* ctx, const float* xyz, int64_t m, rst_target** out) {
  if (!ctx || !out || m < 0 || (m > 0 && !xyz)) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  float* d = nullptr;
  RST_CHECK(upload_xyz(ctx, xyz, m, &d));
  int s = target_build_device(ctx, d, m, true, out);
  free_xyz(ctx, d, m);
  return s;
}

int rst_target_build_device(rst_ctx* ctx, const float* d_xyz, int64_t m, rst_target** out) {
  if (!ctx) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return target_build_device(ctx, d_xyz, m, true, out);
}

int rst_target_free(rst_target* t) {
  if (!t) return RST_OK;
  // blocks go back to the context's pool (no device-wide sync); once the
  // context is gone, to the device
  rst_ctx* ctx = t->ctx;
  if (ctx) {
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    auto& lv = ctx->live;
    for (size_t k = 0; k < lv.size(); ++k)
      if (lv[k] == t) {
        lv[k] = lv.back();
        lv.pop_back();
        break;
      }
    hipSetDevice(ctx->device);
  }
  for (auto& a : t->allocs) ctx_release(ctx, a.first, a.second);
  delete t;
  return RST_OK;
}

int64_t rst_target_size(const rst_target* t) { return t ? t->m : -1; }

int rst_target_compute_normals(rst_ctx* ctx, rst_target* t, int k, const float vp[3]) {
  if (!ctx || !t) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  RST_CHECK(compute_normals(ctx, t, k, vp));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return RST_OK;
}

int rst_target_compute_grid_normals(rst_ctx* ctx, rst_target* t, int radius, const float vp[3]) {
  if (!ctx || !t) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  RST_CHECK(compute_grid_normals(ctx, t, radius, vp));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return RST_OK;
}

int rst_target_get_normals(rst_ctx* ctx, const rst_target* t, float* normals) {
  if (!ctx || !t || (t->m > 0 && !normals)) return RST_E_ARG;
  if (!t->nrm) return RST_E_STATE;
  if (t->m == 0) return RST_OK;
  std::vector<float4> pts(t->m), nrm(t->m);
  RST_HIP(hipMemcpyAsync(pts.data(), t->pts, sizeof(float4) * t->m, hipMemcpyDeviceToHost,
                         ctx->stream));
  RST_HIP(hipMemcpyAsync(nrm.data(), t->nrm, sizeof(float4) * t->m, hipMemcpyDeviceToHost,
                         ctx->stream));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  for (int64_t i = 0; i < t->m; ++i) {
    int j;
    memcpy(&j, &pts[i].w, sizeof(int));
    normals[3 * (int64_t)j + 0] = nrm[i].x;
    normals[3 * (int64_t)j + 1] = nrm[i].y;
    normals[3 * (int64_t)j + 2] = nrm[i].z;
  }
  return RST_OK;
}

int rst_target_query_nn_device(rst_ctx* ctx, const rst_target* t, const float* d_q, int64_t nq,
                               int32_t* d_idx, float* d_d2) {
  if (!ctx || !t || nq < 0 || (nq > 0 && (!d_q || !d_idx || !d_d2))) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return query_nn_device(ctx, t, d_q, nq, d_idx, d_d2);
}

int rst_target_query_nn(rst_ctx* ctx, const rst_target* t, const float* q, int64_t nq,
                        int32_t* idx, float* d2) {
  if (!ctx || !t || nq < 0 || (nq > 0 && (!q || !idx || !d2))) return RST_E_ARG;
  if (nq == 0) return RST_OK;
  RST_HIP(hipSetDevice(ctx->device));
  float* dq = nullptr;
  RST_CHECK(upload_xyz(ctx, q, nq, &dq));
  void* dout = nullptr;
  int s = ctx_workspace(ctx, (sizeof(int32_t) + sizeof(float)) * nq, &dout);
  if (s >= 0) s = query_nn_device(ctx, t, dq, nq, (int32_t*)dout, (float*)((int32_t*)dout + nq));
  if (s >= 0) {
    if (hipMemcpyAsync(idx, dout, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(d2, (int32_t*)dout + nq, sizeof(float) * nq, hipMemcpyDeviceToHost,
                       ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      s = RST_E_HIP;
  }
  free_xyz(ctx, dq, nq);
  return s < 0 ? s : RST_OK;
}

int rst_target_query_nn_warm(rst_ctx* ctx, const rst_target* t, const float* q, int64_t nq,
                             const int32_t* warm, int32_t* idx, float* d2) {
  return rst_debug_query_nn_warm_stats(ctx, t, q, nq, warm, idx, d2, nullptr);
}

int rst_debug_query_nn_warm_stats(rst_ctx* ctx, const rst_target* t, const float* q, int64_t nq,
                                  const int32_t* warm, int32_t* idx, float* d2, int32_t* stats) {
  if (!ctx || !t || nq < 0 || (nq > 0 && (!q || !idx || !d2))) return RST_E_ARG;
  if (nq == 0) return RST_OK;
  RST_HIP(hipSetDevice(ctx->device));
  float* dq = nullptr;
  RST_CHECK(upload_xyz(ctx, q, nq, &dq));
  void* dout = nullptr;
  const int64_t nwav = (nq + 63) / 64;
  int s = ctx_workspace(ctx, (2 * sizeof(int32_t) + sizeof(float)) * nq + 32 * nwav + 256, &dout);
  int32_t* dwarm = nullptr;
  int* dstats = stats ? (int*)((int32_t*)dout + 3 * nq + 16) : nullptr;
  if (s >= 0 && warm) {
    dwarm = (int32_t*)dout + 2 * nq;
    if (hipMemcpyAsync(dwarm, warm, sizeof(int32_t) * nq, hipMemcpyHostToDevice, ctx->stream) !=
        hipSuccess)
      s = RST_E_HIP;
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (stats && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) s = RST_E_HIP;
  if (s >= 0 && e0) s = hipEventRecord(e0, ctx->stream) == hipSuccess ? s : RST_E_HIP;
  if (s >= 0)
    s = query_nn_warm_device(ctx, t, dq, nq, dwarm, (int32_t*)dout, (float*)((int32_t*)dout + nq),
                             dstats);
  if (s >= 0 && e1) s = hipEventRecord(e1, ctx->stream) == hipSuccess ? s : RST_E_HIP;
  if (s >= 0 && stats &&
      hipMemcpyAsync(stats, dstats, 32 * nwav, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    s = RST_E_HIP;
  if (s >= 0) {
    if (hipMemcpyAsync(idx, dout, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(d2, (int32_t*)dout + nq, sizeof(float) * nq, hipMemcpyDeviceToHost,
                       ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      s = RST_E_HIP;
  }
  hipStreamSynchronize(ctx->stream);
  if (e0 && e1 && s >= 0) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) {
      ctx->last_kernel_ms = ms;
      ctx->last_kernel_launches = 1;
    }
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  free_xyz(ctx, dq, nq);
  return s < 0 ? s : RST_OK;
}

int rst_debug_query_nn_fallback(rst_ctx* ctx, const rst_target* t, const float* q, int64_t nq,
                                const int32_t* warm, int mode, int32_t* idx, float* d2,
                                int32_t* path) {
  if (!ctx || !t || nq < 0 || (nq > 0 && (!q || !idx || !d2 || !path))) return RST_E_ARG;
  if (mode != 0 && mode != 2 && mode != 3 && mode != 23 && (mode < 100 || mode > 102) &&
      mode != 1000)
    return RST_E_ARG;
  if (nq == 0) return RST_OK;
  if (t->m == 0) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  float* dq = nullptr;
  RST_CHECK(upload_xyz(ctx, q, nq, &dq));
  void* dout = nullptr;
  int s = ctx_workspace(ctx, (3 * sizeof(int32_t) + sizeof(float)) * nq + 256, &dout);
  int32_t* dwarm = nullptr;
  int32_t* di = (int32_t*)dout;
  float* dd = (float*)(di + nq);
  int32_t* dp = (int32_t*)(dd + nq);
  if (s >= 0 && warm) {
    dwarm = dp + nq;
    if (hipMemcpyAsync(dwarm, warm, sizeof(int32_t) * nq, hipMemcpyHostToDevice, ctx->stream) !=
        hipSuccess)
      s = RST_E_HIP;
  }
  if (s >= 0) s = query_nn_fallback_device(ctx, t, dq, nq, dwarm, mode, di, dd, dp);
  if (s >= 0 &&
      (hipMemcpyAsync(idx, di, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
       hipMemcpyAsync(d2, dd, sizeof(float) * nq, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
       hipMemcpyAsync(path, dp, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
       hipStreamSynchronize(ctx->stream) != hipSuccess))
    s = RST_E_HIP;
  free_xyz(ctx, dq, nq);
  return s < 0 ? s : RST_OK;
}

int rst_debug_target_leaves(rst_ctx* ctx, const rst_target* t, int32_t* lstart, int32_t cap,
                            int32_t* pleaf, int32_t* nleaves) {
  if (!ctx || !t || !nleaves || !t->has_bvh) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  *nleaves = t->nleaves;
  if (lstart && cap >= t->nleaves + 1) {
    RST_HIP(hipMemcpyAsync(lstart, t->lstart, sizeof(int32_t) * (t->nleaves + 1),
                           hipMemcpyDeviceToHost, ctx->stream));
  }
  if (pleaf && t->m > 0)
    RST_HIP(hipMemcpyAsync(pleaf, t->pleaf, sizeof(int32_t) * t->m, hipMemcpyDeviceToHost,
                           ctx->stream));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  return RST_OK;
}

int rst_debug_stream_copy(rst_ctx* ctx, int64_t bytes, int reps, double* gbps) {
  if (!ctx || !gbps || bytes < 16 || reps < 1) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  const int64_t n4 = bytes / 16;
  float4 *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, 16 * n4) != hipSuccess) return RST_E_NOMEM;
  if (hipMalloc(&b, 16 * n4) != hipSuccess) {
    (void)hipFree(a);
    return RST_E_NOMEM;
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int s = RST_OK;
  if (hipMemsetAsync(a, 0, 16 * n4, ctx->stream) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    s = RST_E_HIP;
  float best = 0.f;
  for (int r = 0; r < reps * 6 && s >= 0; ++r) {
    if (hipEventRecord(e0, ctx->stream) != hipSuccess) s = RST_E_HIP;
    switch (r % 6) {  // (variants interleaved: each gets reps launches)
      case 0: k_stream_copy<1, true><<<8192, 256, 0, ctx->stream>>>(a, b, n4); break;
      case 1: k_stream_copy<4, true><<<2048, 256, 0, ctx->stream>>>(a, b, n4); break;
      case 2: k_stream_copy<4, false><<<2048, 256, 0, ctx->stream>>>(a, b, n4); break;
      case 3: k_stream_copy<8, true><<<1024, 256, 0, ctx->stream>>>(a, b, n4); break;
      case 4: k_stream_copy<4, true><<<4096, 256, 0, ctx->stream>>>(a, b, n4); break;
      default: k_stream_copy<2, false><<<8192, 256, 0, ctx->stream>>>(a, b, n4); break;
    }
    if (s >= 0 && (hipGetLastError() != hipSuccess || hipEventRecord(e1, ctx->stream) != hipSuccess ||
                   hipEventSynchronize(e1) != hipSuccess))
      s = RST_E_HIP;
    float ms = 0.f;
    if (s >= 0 && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0.f &&
        (best == 0.f || ms < best))
      best = ms;
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipFree(a);
  (void)hipFree(b);
  if (s < 0) return s;
  *gbps = best > 0.f ? 2.0 * 16.0 * (double)n4 / (best * 1e-3) / 1e9 : 0.0;
  return RST_OK;
}

int rst_debug_launch_rate(rst_ctx* ctx, int nstreams, int launches, int blocks, int threads,
                          double* per_s) {
  if (!ctx || !per_s || nstreams < 1 || nstreams > 64 || launches < 1 || blocks < 1 ||
      threads < 1 || threads > 1024)
    return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  std::vector<hipStream_t> ss(nstreams, nullptr);
  int s = RST_OK;
  for (auto& q : ss)
    if (hipStreamCreateWithFlags(&q, hipStreamNonBlocking) != hipSuccess) s = RST_E_HIP;
  int* sink = nullptr;
  if (s >= 0 && hipMalloc(&sink, sizeof(int) * blocks) != hipSuccess) s = RST_E_NOMEM;
  // warm-up, then the timed round: launches per stream, streams interleaved
  for (int rep = 0; rep < 2 && s >= 0; ++rep) {
    const int nl = rep == 0 ? 8 : launches;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < nl; ++i)
      for (auto q : ss) k_nop<<<blocks, threads, 0, q>>>(sink, 1);
    for (auto q : ss)
      if (hipStreamSynchronize(q) != hipSuccess) s = RST_E_HIP;
    const double dt =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *per_s = (double)nl * nstreams / dt;
  }
  for (auto q : ss)
    if (q) (void)hipStreamDestroy(q);
  if (sink) (void)hipFree(sink);
  return s;
}

int rst_debug_timeline(rst_ctx* ctx, uint64_t* out, int32_t cap, int32_t* iters) {
  if (!ctx || !iters || (cap > 0 && !out)) return RST_E_ARG;
#if RST_TIMELINE
  RST_HIP(hipSetDevice(ctx->device));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  const int n = std::min<int>(cap, kQTrace * kTlKernels * 2);
  memcpy(out, &ctx->h_state->tl[0][0][0], sizeof(uint64_t) * (size_t)std::max(n, 0));
  *iters = ctx->h_state->iter;
  return RST_OK;
#else
  (void)out;
  (void)cap;
  return RST_E_STATE;
#endif
}

int rst_debug_kernel_overlap(rst_ctx* ctx, int nstreams, int launches, int blocks, int threads,
                             int spin_us, int lds_bytes, double* overlap) {
  if (!ctx || !overlap || nstreams < 1 || nstreams > 64 || launches < 1 || blocks < 1 ||
      threads < 1 || threads > 1024 || spin_us < 1 || lds_bytes < 0 || lds_bytes > 160 * 1024)
    return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  std::vector<hipStream_t> ss(nstreams, nullptr);
  int s = RST_OK;
  for (auto& q : ss)
    if (hipStreamCreateWithFlags(&q, hipStreamNonBlocking) != hipSuccess) s = RST_E_HIP;
  int* sink = nullptr;
  if (s >= 0 && hipMalloc(&sink, sizeof(int) * blocks) != hipSuccess) s = RST_E_NOMEM;
  if (s >= 0 && lds_bytes > 64 * 1024 &&
      hipFuncSetAttribute((const void*)k_spin, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) !=
          hipSuccess)
    s = RST_E_HIP;
  const int ticks = spin_us * 100;  // s_memrealtime: 100 MHz
  for (int rep = 0; rep < 2 && s >= 0; ++rep) {
    const int nl = rep == 0 ? 4 : launches;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < nl; ++i)
      for (auto q : ss) k_spin<<<blocks, threads, lds_bytes, q>>>(sink, 1, ticks);
    for (auto q : ss)
      if (hipStreamSynchronize(q) != hipSuccess) s = RST_E_HIP;
    const double dt =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // kernels running at once, on average: their busy time over the wall time
    *overlap = (double)nl * nstreams * spin_us * 1e-6 / dt;
  }
  for (auto q : ss)
    if (q) (void)hipStreamDestroy(q);
  if (sink) (void)hipFree(sink);
  return s;
}

int rst_debug_seq_sum(rst_ctx* ctx, const float* xyzw, int64_t n, int serial, int reps,
                      float out[4], float* ms, int32_t* stats) {
  if (!ctx || !out || n < 0 || (n > 0 && !xyzw) || reps < 1) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  void* d = nullptr;
  const size_t xb = (sizeof(float4) * (size_t)std::max<int64_t>(n, 1) + 255) & ~(size_t)255;
  const size_t bytes = xb + 256 + 256 + seqsum_bytes(n);
  if (hipMalloc(&d, bytes) != hipSuccess) return RST_E_NOMEM;
  float* dout = (float*)((char*)d + xb);
  int* dstats = (int*)((char*)d + xb + 256);
  void* ws = (char*)d + xb + 512;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int s = RST_OK;
  if (n > 0 && hipMemcpyAsync(d, xyzw, sizeof(float4) * n, hipMemcpyHostToDevice, ctx->stream) !=
                   hipSuccess)
    s = RST_E_HIP;
  if (s >= 0 && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) s = RST_E_HIP;
  if (s >= 0 && hipEventRecord(e0, ctx->stream) != hipSuccess) s = RST_E_HIP;
  // serial: 0 the product's choice by size, 1 k_seq_sum4, 2 the map pipeline
  // at any size, 3 the one-wavefront replay (k_sq_serial) at any size, 4 the
  // one-workgroup-per-chain kernel (k_sq_small) up to its 16384 elements
  const int stages = 7 | (serial == 2 ? kSqForceMaps : serial == 3 ? kSqForceSerial : serial == 4 ? kSqForceSmall : 0);
  if (stats && serial != 1 && hipMemsetAsync(dstats, 0, 256, ctx->stream) != hipSuccess) s = RST_E_HIP;
  for (int r = 0; r < reps && s >= 0; ++r)
    s = serial == 1 ? seq_sum4_device(ctx, (const float4*)d, n, dout)
                    : seqsum_enqueue((const float4*)d, n, 4, ws, dout, ctx->stream,
                                     stats ? dstats : nullptr, stages);
  if (s >= 0 && hipEventRecord(e1, ctx->stream) != hipSuccess) s = RST_E_HIP;
  if (s >= 0 && (hipMemcpyAsync(out, dout, sizeof(float) * 4, hipMemcpyDeviceToHost, ctx->stream) !=
                     hipSuccess ||
                 hipStreamSynchronize(ctx->stream) != hipSuccess))
    s = RST_E_HIP;
  if (s >= 0 && ms) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, e0, e1) != hipSuccess) s = RST_E_HIP;
    *ms = t / (float)reps;
  }
  if (s >= 0 && stats && serial != 1 &&
      hipMemcpy(stats, dstats, sizeof(int) * 64, hipMemcpyDeviceToHost) != hipSuccess)
    s = RST_E_HIP;
  hipStreamSynchronize(ctx->stream);
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  hipFree(d);
  return s;
}

int rst_debug_seq_stages(rst_ctx* ctx, const float* xyzw, int64_t n, int nch, int stages,
                         float out[4], void* ws_out, int64_t ws_bytes, int* failed_stage) {
  if (!ctx || !out || n < 1 || !xyzw || nch < 1 || nch > 4 || !failed_stage) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  *failed_stage = 0;
  const size_t sqb = seqsum_bytes(n);
  if (ws_out && ws_bytes < (int64_t)sqb) return RST_E_ARG;
  void* d = nullptr;
  const size_t xb = (sizeof(float4) * (size_t)n + 255) & ~(size_t)255;
  if (hipMalloc(&d, xb + 256 + sqb) != hipSuccess) return RST_E_NOMEM;
  float* dout = (float*)((char*)d + xb);
  void* ws = (char*)d + xb + 256;
  int s = RST_OK;
  if (hipMemsetAsync(d, 0, xb + 256 + sqb, ctx->stream) != hipSuccess ||
      hipMemcpyAsync(d, xyzw, sizeof(float4) * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    s = RST_E_HIP;
  // one kernel at a time, each checked before the next is launched
  for (int b = 0; b < 3 && s >= 0; ++b) {
    if (!(stages & (1 << b))) continue;
    s = seqsum_enqueue((const float4*)d, n, nch, ws, dout, ctx->stream, nullptr, 1 << b);
    if (s < 0) {
      fprintf(stderr, "[rst] seq stage %d: launch failed: %s\n", b + 1, g_last_error);
    } else {
      const hipError_t e = hipStreamSynchronize(ctx->stream);
      if (e != hipSuccess) {
        fprintf(stderr, "[rst] seq stage %d: execution failed: %s (%s)\n", b + 1, hipGetErrorName(e),
                hipGetErrorString(e));
        s = RST_E_HIP;
      }
    }
    if (s < 0) *failed_stage = b + 1;
  }
  if (s >= 0 && hipMemcpy(out, dout, sizeof(float) * 4, hipMemcpyDeviceToHost) != hipSuccess) s = RST_E_HIP;
  if (s >= 0 && ws_out && hipMemcpy(ws_out, ws, sqb, hipMemcpyDeviceToHost) != hipSuccess) s = RST_E_HIP;
  hipFree(d);
  return s;
}

int64_t rst_debug_seq_ws_bytes(int64_t n) { return (int64_t)seqsum_bytes(std::max<int64_t>(n, 1)); }

int rst_debug_seq_sum4(rst_ctx* ctx, const float* xyzw, int64_t n, float out[4]) {
  return rst_debug_seq_sum(ctx, xyzw, n, 0, 1, out, nullptr, nullptr);
}

int rst_debug_icp_partials(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
                           const rst_icp_opts* opts, const float pose[16], float mu,
                           const float smean[3], int32_t iter, double* out, int32_t* nv) {
  if (!ctx) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return icp_debug_partials(ctx, src, tgt, opts, pose, mu, smean, iter, out, nv);
}

int rst_debug_icp_solve(rst_ctx* ctx, const rst_icp_opts* opts, int64_t n_total,
                        const double* totals, const float smean[3], float pose_inout[16],
                        float* mu_inout, int32_t* iter_inout) {
  if (!ctx) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return icp_debug_solve(ctx, opts, n_total, totals, smean, pose_inout, mu_inout, iter_inout);
}

int rst_debug_slab(rst_ctx* ctx, double* out, int64_t n) {
  if (!ctx || !out || n < 0) return RST_E_ARG;
  if (!ctx->d_slab || (size_t)n * sizeof(double) > ctx->slab_bytes) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  RST_HIP(hipStreamSynchronize(ctx->stream));
  RST_HIP(hipMemcpy(out, ctx->d_slab, sizeof(double) * n, hipMemcpyDeviceToHost));
  return RST_OK;
}

int rst_debug_iter_diag(rst_ctx* ctx, int32_t* out, int32_t n) {
  if (!ctx || !out || n < 0) return RST_E_ARG;
  for (int i = 0; i < n && i < kQTrace; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = ctx->h_state->diag[i][j];
  return RST_OK;
}

int rst_debug_queue_trace(rst_ctx* ctx, int32_t* out, int32_t n) {
  if (!ctx || !out || n < 0) return RST_E_ARG;
  for (int i = 0; i < n && i < kQTrace; ++i) {
    out[5 * i] = ctx->h_state->qlen[i];
    for (int j = 0; j < 4; ++j) out[5 * i + 1 + j] = ctx->h_state->path[i][j];
  }
  return RST_OK;
}

int rst_target_query_knn(rst_ctx* ctx, const rst_target* t, const float* q, int64_t nq, int k,
                         int32_t* idx, float* d2) {
  if (!ctx || !t || nq < 0 || k < 1 || k > 32 || (nq > 0 && (!q || !idx || !d2)))
    return RST_E_ARG;
  if (nq == 0) return RST_OK;
  RST_HIP(hipSetDevice(ctx->device));
  float* dq = nullptr;
  RST_CHECK(upload_xyz(ctx, q, nq, &dq));
  void* dout = nullptr;
  const size_t cnt = (size_t)nq * k;
  int s = ctx_workspace(ctx, (sizeof(int32_t) + sizeof(float)) * cnt, &dout);
  if (s >= 0)
    s = query_knn_device(ctx, t, dq, nq, k, (int32_t*)dout, (float*)((int32_t*)dout + cnt));
  if (s >= 0) {
    if (hipMemcpyAsync(idx, dout, sizeof(int32_t) * cnt, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(d2, (int32_t*)dout + cnt, sizeof(float) * cnt, hipMemcpyDeviceToHost,
                       ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      s = RST_E_HIP;
  }
  free_xyz(ctx, dq, nq);
  return s < 0 ? s : RST_OK;
}

// ---- ICP ---------------------------------------------------------------------------
int rst_icp_align_prepared(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
                           const rst_icp_opts* opts, float pose_inout[16], float* mean_cost,
                           int32_t* iterations_run) {
  if (!ctx || !src || !tgt || !pose_inout) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return icp_align_prepared(ctx, src, tgt, opts, pose_inout, mean_cost, iterations_run, nullptr);
}

int rst_icp_align_prepared_async(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
                                 const rst_icp_opts* opts, const float pose_in[16]) {
  if (!ctx || !src || !tgt || !pose_in) return RST_E_ARG;
  if (ctx->pend.active) return RST_E_STATE;  // one align in flight per context
  RST_HIP(hipSetDevice(ctx->device));
  const int s = icp_launch(ctx, src, tgt, opts, pose_in, nullptr);
  if (s == RST_FALSE) {  // the reference's early false: _wait reports it
    ctx->pend.active = true;
    ctx->pend.early_false = true;
  }
  return s;
}

int rst_icp_align_pyramid_async(rst_ctx* ctx, const rst_target* const* src,
                                const rst_target* const* tgt, int nlevels, const int32_t* iters,
                                const rst_icp_opts* opts, const float pose_in[16]) {
  if (!ctx || !src || !tgt || !iters || !pose_in || nlevels < 1 || nlevels > 16) return RST_E_ARG;
  for (int l = 0; l < nlevels; ++l)
    if (!src[l] || !tgt[l] || iters[l] < 0) return RST_E_ARG;
  if (ctx->pend.active) return RST_E_STATE;
  RST_HIP(hipSetDevice(ctx->device));
  rst_icp_opts o;
  if (opts)
    o = *opts;
  else
    rst_icp_opts_default(&o);
  // level 0 decides the result: its early false (align_icp.cpp:77-79) means
  // nothing to run; _wait reports it with the pose untouched
  if (src[0]->m < 3 || tgt[0]->m < 3 || (o.mode == RST_P2PLANE && src[0]->m < 6)) {
    ctx->pend = {};
    ctx->pend.active = true;
    ctx->pend.early_false = true;
    return RST_FALSE;
  }
  bool chained = false;  // a solve has been enqueued on the context's state
  for (int l = nlevels - 1; l >= 0; --l) {
    o.max_iter = iters[l];
    const int s = icp_launch(ctx, src[l], tgt[l], &o, pose_in, nullptr, chained, l);
    if (s == RST_FALSE) continue;  // early false: the pose passes through (level 0 excluded above)
    if (s != RST_OK) {
      ctx->pend = {};
      hipStreamSynchronize(ctx->stream);
      return s;
    }
    chained = true;
  }
  ctx->pend.pyramid = true;
  return RST_OK;
}

int rst_icp_align_batch_async(rst_ctx* ctx, int32_t nb, const rst_target* const* src,
                              const rst_target* const* tgt, const rst_icp_opts* opts,
                              const float* poses_in) {
  if (!ctx || nb < 1 || !src || !tgt || !poses_in) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return icp_launch_batch(ctx, nb, src, tgt, opts, poses_in);
}

int rst_icp_align_batch_wait(rst_ctx* ctx, float* poses_inout, float* mean_costs, int32_t* status,
                             int32_t* iterations) {
  if (!ctx || !poses_inout || !status) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return icp_finish_batch(ctx, poses_inout, mean_costs, status, iterations);
}

int rst_icp_align_wait(rst_ctx* ctx, float pose_inout[16], float* mean_cost,
                       int32_t* iterations_run) {
  if (!ctx || !pose_inout) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return icp_finish(ctx, pose_inout, mean_cost, iterations_run);
}

int rst_icp_align_device(rst_ctx* ctx, const float* d_src, int64_t n, const rst_target* tgt,
                         const rst_icp_opts* opts, float pose_inout[16], float* mean_cost) {
  if (!ctx || !tgt || !pose_inout || n < 0 || (n > 0 && !d_src)) return RST_E_ARG;
  if (n < 3 || tgt->m < 3) return RST_FALSE;  // align_icp.cpp:77-79
  RST_HIP(hipSetDevice(ctx->device));
  rst_target* s = nullptr;
  RST_CHECK(target_build_device(ctx, d_src, n, false, &s));
  int r = icp_align_prepared(ctx, s, tgt, opts, pose_inout, mean_cost, nullptr, nullptr);
  rst_target_free(s);
  return r;
}

int rst_icp_align(rst_ctx* ctx, const float* src, int64_t n, const rst_target* tgt,
                  const rst_icp_opts* opts, float pose_inout[16], float* mean_cost) {
  if (!ctx || !tgt || !pose_inout || n < 0 || (n > 0 && !src)) return RST_E_ARG;
  if (n < 3 || tgt->m < 3) return RST_FALSE;  // align_icp.cpp:77-79
  RST_HIP(hipSetDevice(ctx->device));
  float* d = nullptr;
  RST_CHECK(upload_xyz(ctx, src, n, &d));
  int r = rst_icp_align_device(ctx, d, n, tgt, opts, pose_inout, mean_cost);
  free_xyz(ctx, d, n);
  return r;
}

int rst_icp_align_clouds(rst_ctx* ctx, const float* src, int64_t n, const float* dst, int64_t m,
                         const rst_icp_opts* opts, float pose_inout[16], float* mean_cost) {
  if (!ctx || !pose_inout || n < 0 || m < 0 || (n > 0 && !src) || (m > 0 && !dst))
    return RST_E_ARG;
  if (n < 3 || m < 3) return RST_FALSE;  // align_icp.cpp:77-79
  rst_target* t = nullptr;
  RST_CHECK(rst_target_build(ctx, dst, m, &t));  // :165 KDTree3f{dst,16}
  int r = rst_icp_align(ctx, src, n, t, opts, pose_inout, mean_cost);
  rst_target_free(t);
  return r;
}

int rst_kabsch_solve(rst_ctx* ctx, const double cov[9], const float smean[3],
                     const float dmean[3], float pose_out[16]) {
  if (!ctx || !cov || !smean || !dmean || !pose_out) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return kabsch_device(ctx, cov, smean, dmean, pose_out);
}

int rst_solve_kabsch(rst_ctx* ctx, const float* src, int64_t n, const float* dst, int64_t m,
                     const int32_t* pairs, const float* weights, int64_t k, float pose_out[16]) {
  if (!ctx || !pose_out || n < 0 || m < 0 || k < 0 || (n > 0 && !src) || (m > 0 && !dst) ||
      (k > 0 && !pairs))
    return RST_E_ARG;
  if (n < 3 || m < 3) return RST_FALSE;  // align_icp.cpp:22-24, pose untouched
  if (k == 0) {
    // the reference with no correspondences: means 0/0 = NaN (:33-34), an
    // all-zero covariance whose Jacobi SVD is U = V = I, so R = I and
    // t = dst_mean - R src_mean = NaN; it returns true (:69-70)
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 4; ++r) pose_out[c * 4 + r] = (r == c) ? 1.0f : 0.0f;
    for (int r = 0; r < 3; ++r) pose_out[12 + r] = NAN;
    return RST_OK;
  }
  for (int64_t c = 0; c < k; ++c)        // host-side bounds check before any launch
    if (pairs[2 * c] < 0 || pairs[2 * c] >= n || pairs[2 * c + 1] < 0 || pairs[2 * c + 1] >= m)
      return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  float *ds = nullptr, *dd = nullptr;
  RST_CHECK(upload_xyz(ctx, src, n, &ds));
  int r = upload_xyz(ctx, dst, m, &dd);
  // pairs + weights through the pinned staging buffer into the workspace
  const size_t pb = sizeof(int32_t) * 2 * (size_t)k, wb = weights ? sizeof(float) * (size_t)k : 0;
  const size_t pwb = (pb + wb + 255) & ~(size_t)255;
  void* ws = nullptr;
  if (r >= 0) r = ctx_workspace(ctx, pwb + solve_kabsch_ws_bytes(k), &ws);
  if (r >= 0) r = stage_h2d(ctx, ws, pairs, pb);
  if (r >= 0 && weights) r = stage_h2d(ctx, (char*)ws + pb, weights, wb);
  if (r >= 0)
    r = solve_kabsch_device(ctx, ds, dd, (const int32_t*)ws,
                            weights ? (const float*)((char*)ws + pb) : nullptr, k,
                            (char*)ws + pwb, pose_out);
  free_xyz(ctx, dd, m);
  free_xyz(ctx, ds, n);
  return r;
}

// ComputeCentroid (point_cloud_utils.cpp:92-98): the fp32 sequential sums in
// input order (seqsum.hip, bit-exact), times float(1.0 / n)
int rst_compute_centroid(rst_ctx* ctx, const float* xyz, int64_t n, float out[3]) {
  if (!ctx || !out || n <= 0 || !xyz) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  float* d = nullptr;
  RST_CHECK(upload_xyz(ctx, xyz, n, &d));
  void* ws = nullptr;
  int r = ctx_workspace(ctx, centroid_ws_bytes(n), &ws);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (r >= 0) r = centroid_seq_device(ctx, d, n, ws, s);
  free_xyz(ctx, d, n);
  if (r < 0) return r;
  const float f = (float)(1.0 / (double)n);  // Vector3f *= double: the float Scalar
  for (int k = 0; k < 3; ++k) out[k] = s[k] * f;
  return RST_OK;
}

}  // extern "C"
