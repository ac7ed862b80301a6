// synth.cpp -- synthetic frame source (rs_tracker/driver decoupled from the
// camera).  Stands in for the RealSense pipeline behind DataSource<Derived>
// (data_source.hpp:9-41) and RandomSource (data_source.hpp:22-41).
//
// Scene: a closed room (walls) with seeded spheres and yaw-rotated boxes, so
// every frame is non-planar (no Kabsch degeneracy).  Depth is z along the
// optical axis, ray-cast through the same pinhole model the unprojection
// inverts, perturbed by Gaussian noise, quantised to depth units, with a
// seeded fraction of pixels dropped to 0 (the RealSense "no data" value).
// Host code; deterministic in (scene seed, noise seed).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "rst_align.h"

namespace {

inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t hash3(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t s = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full ^
               (c + 0x165667B19E3779F9ull);
  return splitmix64(s);
}
inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

struct Sphere {
  double c[3], r;
};
struct Box {
  double c[3], h[3], yaw;
};

}  // namespace

struct rst_scene {
  double room_lo[3], room_hi[3];
  std::vector<Sphere> spheres;
  std::vector<Box> boxes;
};

namespace {

// nearest positive hit along o + t d (t in camera z units)
double trace(const rst_scene& s, const double o[3], const double d[3]) {
  double best = INFINITY;
  for (int a = 0; a < 3; ++a) {  // room: camera inside, exit distance
    if (d[a] > 1e-12) best = std::fmin(best, (s.room_hi[a] - o[a]) / d[a]);
    if (d[a] < -1e-12) best = std::fmin(best, (s.room_lo[a] - o[a]) / d[a]);
  }
  for (const Sphere& sp : s.spheres) {
    const double oc[3] = {o[0] - sp.c[0], o[1] - sp.c[1], o[2] - sp.c[2]};
    const double A = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const double B = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
    const double C = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - sp.r * sp.r;
    const double disc = B * B - A * C;
    if (disc < 0) continue;
    const double sq = std::sqrt(disc);
    double t = (-B - sq) / A;
    if (t <= 1e-9) t = (-B + sq) / A;
    if (t > 1e-9 && t < best) best = t;
  }
  for (const Box& b : s.boxes) {
    const double cy = std::cos(b.yaw), sy = std::sin(b.yaw);
    // world -> box frame: rotate by -yaw about y
    const double ow[3] = {o[0] - b.c[0], o[1] - b.c[1], o[2] - b.c[2]};
    const double ob[3] = {cy * ow[0] - sy * ow[2], ow[1], sy * ow[0] + cy * ow[2]};
    const double db[3] = {cy * d[0] - sy * d[2], d[1], sy * d[0] + cy * d[2]};
    double tn = -INFINITY, tf = INFINITY;
    bool miss = false;
    for (int a = 0; a < 3 && !miss; ++a) {
      if (std::fabs(db[a]) < 1e-15) {
        if (ob[a] < -b.h[a] || ob[a] > b.h[a]) miss = true;
        continue;
      }
      double t1 = (-b.h[a] - ob[a]) / db[a], t2 = (b.h[a] - ob[a]) / db[a];
      if (t1 > t2) std::swap(t1, t2);
      tn = std::fmax(tn, t1);
      tf = std::fmin(tf, t2);
      if (tn > tf) miss = true;
    }
    if (!miss && tf > 1e-9) {
      const double t = tn > 1e-9 ? tn : tf;
      if (t < best) best = t;
    }
  }
  return best;
}

void euler_pose(double yaw, double pitch, double roll, const double c[3], float T[16]) {
  // R = Ry(yaw) Rx(pitch) Rz(roll), column-major 4x4 camera->world
  const double cy = std::cos(yaw), sy = std::sin(yaw), cp = std::cos(pitch), sp = std::sin(pitch),
               cr = std::cos(roll), sr = std::sin(roll);
  const double Ry[9] = {cy, 0, -sy, 0, 1, 0, sy, 0, cy};  // col-major
  const double Rx[9] = {1, 0, 0, 0, cp, sp, 0, -sp, cp};
  const double Rz[9] = {cr, sr, 0, -sr, cr, 0, 0, 0, 1};
  double M[9], R[9];
  for (int cc = 0; cc < 3; ++cc)
    for (int r = 0; r < 3; ++r) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += Ry[k * 3 + r] * Rx[cc * 3 + k];
      M[cc * 3 + r] = s;
    }
  for (int cc = 0; cc < 3; ++cc)
    for (int r = 0; r < 3; ++r) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += M[k * 3 + r] * Rz[cc * 3 + k];
      R[cc * 3 + r] = s;
    }
  for (int cc = 0; cc < 3; ++cc) {
    for (int r = 0; r < 3; ++r) T[cc * 4 + r] = (float)R[cc * 3 + r];
    T[cc * 4 + 3] = 0.f;
  }
  for (int r = 0; r < 3; ++r) T[12 + r] = (float)c[r];
  T[15] = 1.f;
}

}  // namespace

extern "C" {

int rst_scene_create(uint64_t seed, rst_scene** out) {
  if (!out) return RST_E_ARG;
  rst_scene* s = new rst_scene();
  const double lo[3] = {-2.0, -1.5, -1.0}, hi[3] = {2.0, 1.5, 4.5};
  memcpy(s->room_lo, lo, sizeof(lo));
  memcpy(s->room_hi, hi, sizeof(hi));
  uint64_t st = seed * 0x2545F4914F6CDD1Dull + 12345;
  auto U = [&](double a, double b) { return a + (b - a) * u01(splitmix64(st)); };
  for (int i = 0; i < 8; ++i) {
    Sphere sp;
    sp.c[0] = U(-1.5, 1.5);
    sp.c[1] = U(-1.1, 1.1);
    sp.c[2] = U(1.3, 3.8);
    sp.r = U(0.15, 0.45);
    s->spheres.push_back(sp);
  }
  for (int i = 0; i < 5; ++i) {
    Box b;
    b.c[0] = U(-1.5, 1.5);
    b.c[1] = U(-1.0, 1.2);
    b.c[2] = U(1.5, 4.0);
    b.h[0] = U(0.1, 0.4);
    b.h[1] = U(0.1, 0.5);
    b.h[2] = U(0.1, 0.4);
    b.yaw = U(-0.8, 0.8);
    s->boxes.push_back(b);
  }
  *out = s;
  return RST_OK;
}

int rst_scene_destroy(rst_scene* s) {
  delete s;
  return RST_OK;
}

int rst_scene_render_depth(const rst_scene* s, const float T[16], const rst_intrinsics* K,
                           uint64_t noise_seed, float noise_sigma, float invalid_frac,
                           uint16_t* depth) {
  if (!s || !T || !K || !depth || K->width <= 0 || K->height <= 0 || !(K->depth_scale > 0))
    return RST_E_ARG;
  const double o[3] = {T[12], T[13], T[14]};
  const double zmin = K->min_depth > 0 ? K->min_depth : 0.0;
  const double zmax = K->max_depth > 0 ? K->max_depth : 1e30;
  for (int v = 0; v < K->height; ++v) {
    for (int u = 0; u < K->width; ++u) {
      const double dc[3] = {((double)u - K->cx) / K->fx, ((double)v - K->cy) / K->fy, 1.0};
      double dw[3];
      for (int r = 0; r < 3; ++r)
        dw[r] = T[0 * 4 + r] * dc[0] + T[1 * 4 + r] * dc[1] + T[2 * 4 + r] * dc[2];
      double z = trace(*s, o, dw);  // parameter t == camera z (dc.z == 1)
      const uint64_t pix = (uint64_t)v * K->width + u;
      const uint64_t h1 = hash3(noise_seed, pix, 1), h2 = hash3(noise_seed, pix, 2),
                     h3 = hash3(noise_seed, pix, 3);
      if (noise_sigma > 0) {
        const double a = std::fmax(u01(h1), 1e-300), b = u01(h2);
        z += noise_sigma * std::sqrt(-2.0 * std::log(a)) * std::cos(2.0 * M_PI * b);
      }
      uint16_t d = 0;
      if (std::isfinite(z) && z >= zmin && z <= zmax && u01(h3) >= invalid_frac) {
        const double q = std::floor(z / K->depth_scale + 0.5);
        d = (uint16_t)(q < 1 ? 0 : (q > 65535 ? 65535 : q));
      }
      depth[pix] = d;
    }
  }
  return RST_OK;
}

int rst_scene_trajectory(const rst_scene* s, int32_t frame, float T[16]) {
  if (!s || !T) return RST_E_ARG;
  // ~30 fps hand-held motion: peak ~0.6 m/s and ~45 deg/s, i.e. 1-3 cm and
  // about 1-2 degrees between consecutive frames
  const double tau = frame / 30.0;
  const double c[3] = {0.5 * std::sin(1.2 * tau), 0.15 * std::sin(1.7 * tau + 0.5),
                       0.4 * std::sin(0.9 * tau)};
  euler_pose(0.5 * std::sin(1.5 * tau), 0.2 * std::sin(2.1 * tau), 0.1 * std::sin(1.3 * tau), c,
             T);
  return RST_OK;
}

int rst_random_cloud(uint64_t seed, int64_t n, float* xyz) {
  if (n < 0 || (n > 0 && !xyz)) return RST_E_ARG;
  uint64_t st = seed ^ 0xD1B54A32D192ED03ull;
  for (int64_t i = 0; i < 3 * n; ++i) xyz[i] = (float)(2.0 * u01(splitmix64(st)) - 1.0);
  return RST_OK;
}

}  // extern "C"
