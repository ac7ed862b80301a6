// unproject.hip -- depth (u16) -> xyz, the step librealsense's
// rs2::pointcloud::calculate does for the reference (data_source_rs.cpp:89-90,
// rs_driver.cpp:201-202), followed by the reference's NaN->0 copy
// (data_source_rs.cpp:34-41) or, by default, an order-preserving compaction
// that drops invalid pixels.
//
// Pinhole deprojection with rs2_deproject_pixel_to_point's op order (no
// distortion):  x = (u - ppx)/fx,  y = (v - ppy)/fy,  P = (z*x, z*y, z).
// HBM traffic: 2 B/px in, 12 B/valid px out (+ 4 B per 1024-px tile count).
//
// Pyramid levels (BASELINE configs[4]): level l reads every s = 2^l-th pixel
// of every s-th row -- pixel (u, v) = (s*ul, s*vl) of the full image with
// the full image's intrinsics, so a level's points are exactly a subset of
// the level-0 points (2 B / s^2 px in).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rst_device.hpp"
#include "rst_internal.hpp"

namespace rst {
namespace {

constexpr int kBS = 256;
constexpr int kRounds = 4;
constexpr int kTile = kBS * kRounds;

struct Cam {
  float fx, fy, cx, cy, scale, zmin, zmax;
  int w;       // width of the (decimated) pixel grid
  int s;       // decimation stride (1 = full resolution)
  int64_t ws;  // row pitch of the depth image (pixels)
};

// depth index of grid pixel p
__device__ __forceinline__ int64_t src_px(int64_t p, const Cam& c) {
  return (p / c.w) * c.s * c.ws + (p % c.w) * c.s;
}

__device__ __forceinline__ bool valid_px(uint16_t d, const Cam& c, float& z) {
  z = c.scale * (float)d;
  return d != 0 && (c.zmin <= 0.f || z >= c.zmin) && (c.zmax <= 0.f || z <= c.zmax);
}

__global__ __launch_bounds__(kBS) void k_count(const uint16_t* __restrict__ depth, int64_t npx,
                                               Cam c, uint32_t* __restrict__ counts) {
  __shared__ uint32_t s[kBS / kWave];
  uint32_t cnt = 0;
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int64_t p = base + r * kBS + threadIdx.x;
    float z;
    if (p < npx && valid_px(depth[src_px(p, c)], c, z)) ++cnt;
  }
  // wave + block sum
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

__global__ __launch_bounds__(kBS) void k_write(const uint16_t* __restrict__ depth, int64_t npx,
                                               Cam c, int keep_invalid,
                                               const uint32_t* __restrict__ offsets,
                                               float* __restrict__ xyz,
                                               int32_t* __restrict__ pixmap) {
  __shared__ uint32_t wtot[kBS / kWave];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t run = keep_invalid ? 0u : offsets[blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * kTile;
  for (int r = 0; r < kRounds; ++r) {
    const int64_t p = base + r * kBS + threadIdx.x;
    const bool inb = p < npx;
    const uint16_t d = inb ? depth[src_px(p, c)] : (uint16_t)0;
    float z;
    const bool ok = inb && valid_px(d, c, z);
    const int u = (int)(p % c.w) * c.s, v = (int)(p / c.w) * c.s;
    const float x = ((float)u - c.cx) / c.fx;
    const float y = ((float)v - c.cy) / c.fy;
    if (keep_invalid) {
      if (inb) {
        xyz[3 * p + 0] = ok ? z * x : 0.f;
        xyz[3 * p + 1] = ok ? z * y : 0.f;
        xyz[3 * p + 2] = ok ? z : 0.f;
      }
      continue;
    }
    const uint64_t bal = __ballot(ok);
    if (lane == 0) wtot[w] = __popcll(bal);
    __syncthreads();
    uint32_t off = run;
    for (int k = 0; k < w; ++k) off += wtot[k];
    if (ok) {
      const int64_t o = off + __popcll(bal & lt);
      xyz[3 * o + 0] = z * x;
      xyz[3 * o + 1] = z * y;
      xyz[3 * o + 2] = z;
    }
    if (pixmap && inb) pixmap[p] = ok ? (int32_t)(off + __popcll(bal & lt)) : -1;
    uint32_t tot = 0;
    for (int k = 0; k < kBS / kWave; ++k) tot += wtot[k];
    run += tot;
    __syncthreads();
  }
}

// pixel map: original point index -> sorted position of the built target;
// the grid's points in pixel order (PixView::pts)
__global__ __launch_bounds__(kBS) void k_pixmap_sorted(int32_t* __restrict__ map, int64_t npx,
                                                       const int32_t* __restrict__ inv,
                                                       const float4* __restrict__ spts,
                                                       float4* __restrict__ ppts) {
  const int64_t p = (int64_t)blockIdx.x * kBS + threadIdx.x;
  if (p < npx) {
    const int32_t o = map[p];
    const int32_t q = o >= 0 ? inv[o] : -1;
    map[p] = q;
    ppts[p] = q >= 0 ? spts[q] : make_float4(NAN, NAN, NAN, __int_as_float(-1));
  }
}

}  // namespace

namespace {
__global__ __launch_bounds__(1024) void k_scan_small(uint32_t* __restrict__ a, int n,
                                                     uint32_t* __restrict__ total) {
  __shared__ uint32_t s[1024];
  const int per = (n + 1023) / 1024;
  const int b = threadIdx.x * per;
  const int e = std::min(b + per, n);
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
}  // namespace

int unproject_device(rst_ctx* ctx, const uint16_t* d_depth, const rst_intrinsics* K,
                     int keep_invalid, float* d_xyz, int64_t* n_out, int stride,
                     int32_t* d_pixmap) {
  if (!ctx || !d_depth || !K || !d_xyz || !n_out) return RST_E_ARG;
  if (K->width <= 0 || K->height <= 0 || !(K->fx != 0.f) || !(K->fy != 0.f)) return RST_E_ARG;
  if (stride < 1 || stride > 1024) return RST_E_ARG;
  const int wl = (K->width + stride - 1) / stride, hl = (K->height + stride - 1) / stride;
  const int64_t npx = (int64_t)wl * hl;
  Cam c{K->fx, K->fy, K->cx, K->cy, K->depth_scale, K->min_depth, K->max_depth, wl, stride,
        (int64_t)K->width};
  const int nb = (int)((npx + kTile - 1) / kTile);
  hipStream_t st = ctx->stream;
  if (keep_invalid) {
    k_write<<<nb, kBS, 0, st>>>(d_depth, npx, c, 1, nullptr, d_xyz, nullptr);
    RST_HIP(hipGetLastError());
    *n_out = npx;
    return RST_OK;
  }
  void* ws = nullptr;
  RST_CHECK(ctx_workspace(ctx, sizeof(uint32_t) * (nb + 64), &ws));
  uint32_t* counts = (uint32_t*)ws;
  uint32_t* total = counts + nb + 16;
  k_count<<<nb, kBS, 0, st>>>(d_depth, npx, c, counts);
  k_scan_small<<<1, 1024, 0, st>>>(counts, nb, total);
  k_write<<<nb, kBS, 0, st>>>(d_depth, npx, c, 0, counts, d_xyz, d_pixmap);
  RST_HIP(hipGetLastError());
  uint32_t h = 0;
  RST_HIP(hipMemcpyAsync(&h, total, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  RST_HIP(hipStreamSynchronize(st));
  *n_out = h;
  return RST_OK;
}

}  // namespace rst

using namespace rst;

extern "C" {

int rst_unproject_device(rst_ctx* ctx, const uint16_t* d_depth, const rst_intrinsics* K,
                         int keep_invalid, float* d_xyz_out, int64_t* n_out) {
  if (!ctx) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return unproject_device(ctx, d_depth, K, keep_invalid, d_xyz_out, n_out, 1);
}

int rst_unproject_strided_device(rst_ctx* ctx, const uint16_t* d_depth, const rst_intrinsics* K,
                                 int stride, int keep_invalid, float* d_xyz_out, int64_t* n_out) {
  if (!ctx) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return unproject_device(ctx, d_depth, K, keep_invalid, d_xyz_out, n_out, stride);
}

int rst_unproject(rst_ctx* ctx, const uint16_t* depth, const rst_intrinsics* K, int keep_invalid,
                  float* xyz_out, int64_t* n_out) {
  if (!ctx || !depth || !K || !xyz_out || !n_out) return RST_E_ARG;
  if (K->width <= 0 || K->height <= 0) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  const int64_t npx = (int64_t)K->width * K->height;
  uint16_t* dd = nullptr;
  float* dx = nullptr;
  if (hipMalloc(&dd, sizeof(uint16_t) * npx) != hipSuccess) return RST_E_NOMEM;
  if (hipMalloc(&dx, sizeof(float) * 3 * npx) != hipSuccess) {
    hipFree(dd);
    return RST_E_NOMEM;
  }
  int s = RST_OK;
  if (hipMemcpyAsync(dd, depth, sizeof(uint16_t) * npx, hipMemcpyHostToDevice, ctx->stream) !=
      hipSuccess)
    s = RST_E_HIP;
  int64_t n = 0;
  if (s >= 0) s = unproject_device(ctx, dd, K, keep_invalid, dx, &n, 1);
  if (s >= 0) {
    if (hipMemcpyAsync(xyz_out, dx, sizeof(float) * 3 * n, hipMemcpyDeviceToHost, ctx->stream) !=
            hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      s = RST_E_HIP;
    *n_out = n;
  }
  hipStreamSynchronize(ctx->stream);
  hipFree(dd);
  hipFree(dx);
  return s;
}

}  // extern "C"

namespace rst {
// depth (device) -> points of pyramid level `stride` -> target handle
// (+ normals: normals_k > 0 kNN-PCA, < 0 image-grid window of radius -normals_k)
static int frame_prepare(rst_ctx* ctx, const uint16_t* d_depth, const rst_intrinsics* K,
                         int stride, int normals_k, rst_target** out) {
  const int64_t npx = (int64_t)K->width * K->height;
  if (stride < 1) return RST_E_ARG;
  const int wl = (K->width + stride - 1) / stride, hl = (K->height + stride - 1) / stride;
  const int64_t npl = (int64_t)wl * hl;
  float* dx = nullptr;
  size_t dxc = 0, pmc = 0;
  int32_t* pm = nullptr;  // the level's pixel map (the target keeps it)
  float4* pp = nullptr;   // ... and its points in pixel order
  size_t ppc = 0;
  RST_CHECK(ctx_alloc(ctx, sizeof(float) * 3 * std::max<int64_t>(npx, 1), (void**)&dx, &dxc));
  if (ctx_alloc(ctx, sizeof(int32_t) * std::max<int64_t>(npl, 1), (void**)&pm, &pmc) < 0) {
    ctx_release(ctx, dx, dxc);
    return RST_E_NOMEM;
  }
  if (ctx_alloc(ctx, sizeof(float4) * std::max<int64_t>(npl, 1), (void**)&pp, &ppc) < 0) {
    ctx_release(ctx, dx, dxc);
    ctx_release(ctx, pm, pmc);
    return RST_E_NOMEM;
  }
  int64_t n = 0;
  int s = unproject_device(ctx, d_depth, K, 0, dx, &n, stride, pm);
  rst_target* t = nullptr;
  if (s >= 0) s = target_build_device(ctx, dx, n, true, &t);
  if (s >= 0) {
    k_pixmap_sorted<<<(int)((npl + kBS - 1) / kBS), kBS, 0, ctx->stream>>>(pm, npl, t->inv,
                                                                            t->pts, pp);
    t->allocs.emplace_back(pm, pmc);  // freed with the target
    t->allocs.emplace_back(pp, ppc);
    t->pix.map = pm;
    t->pix.pts = pp;
    t->pix.inv = t->inv;
    pm = nullptr;
    pp = nullptr;
    t->pix.fx = K->fx;
    t->pix.fy = K->fy;
    t->pix.cx = K->cx;
    t->pix.cy = K->cy;
    t->pix.w = wl;
    t->pix.h = hl;
    t->pix.s = stride;
  }
  if (s >= 0 && normals_k != 0) {
    const float vp[3] = {0.f, 0.f, 0.f};  // the camera
    s = normals_k > 0 ? compute_normals(ctx, t, normals_k, vp)
                      : compute_grid_normals(ctx, t, -normals_k, vp);
  }
  hipStreamSynchronize(ctx->stream);
  ctx_release(ctx, dx, dxc);
  if (pm) ctx_release(ctx, pm, pmc);
  if (pp) ctx_release(ctx, pp, ppc);
  if (s < 0) {
    if (t) rst_target_free(t);
    return s;
  }
  *out = t;
  return RST_OK;
}
}  // namespace rst

extern "C" {

int rst_frame_prepare_device(rst_ctx* ctx, const uint16_t* d_depth, const rst_intrinsics* K,
                             int normals_k, rst_target** out) {
  if (!ctx || !d_depth || !K || !out) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  return frame_prepare(ctx, d_depth, K, 1, normals_k, out);
}

int rst_frame_prepare_pyramid_device(rst_ctx* ctx, const uint16_t* d_depth,
                                     const rst_intrinsics* K, int nlevels, int normals_k,
                                     rst_target** out_levels) {
  if (!ctx || !d_depth || !K || !out_levels || nlevels < 1 || nlevels > 10) return RST_E_ARG;
  RST_HIP(hipSetDevice(ctx->device));
  for (int l = 0; l < nlevels; ++l) out_levels[l] = nullptr;
  for (int l = 0; l < nlevels; ++l) {
    const int s = frame_prepare(ctx, d_depth, K, 1 << l, normals_k, &out_levels[l]);
    if (s < 0) {
      for (int k = 0; k < l; ++k) {
        rst_target_free(out_levels[k]);
        out_levels[k] = nullptr;
      }
      return s;
    }
  }
  return RST_OK;
}

}  // extern "C"
