// rs_tracker/common/types.hpp -- boundary types of the align module
// (reference: rs_tracker/common/include/rs_tracker/common/types.hpp:11-20)
// plus the GPU context the C ABI needs.
//
//   Cloud3f     cho::core::PointCloud<float,3> = Eigen 3 x N column-major
//               float, i.e. AoS xyz (point i at data()[3i..3i+2]).  cho_util
//               is not vendored by the reference, so this is a minimal
//               owner with the same byte layout and the accessors the align
//               code uses (GetNumPoints, GetPoint, GetData-as-pointer).
//   Isometry3f  Eigen::Isometry3f when Eigen is available (the reference's
//               own type), else a 4 x 4 column-major float stand-in with the
//               same matrix() layout.
#pragma once

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "rst_align.h"

#if __has_include(<Eigen/Geometry>)
#include <Eigen/Geometry>
#define RS_TRACKER_HAVE_EIGEN 1
#endif

namespace rs_tracker {

class Cloud3f {
 public:
  Cloud3f() = default;
  explicit Cloud3f(int64_t n) : xyz_(3 * n, 0.f) {}
  Cloud3f(const float* xyz, int64_t n) : xyz_(xyz, xyz + 3 * n) {}

  int64_t cols() const { return (int64_t)xyz_.size() / 3; }
  int64_t GetNumPoints() const { return cols(); }
  bool IsEmpty() const { return xyz_.empty(); }
  void Resize(int64_t n) { xyz_.resize(3 * n); }
  float* data() { return xyz_.data(); }
  const float* data() const { return xyz_.data(); }
  float* GetPoint(int64_t i) { return xyz_.data() + 3 * i; }
  const float* GetPoint(int64_t i) const { return xyz_.data() + 3 * i; }

 private:
  std::vector<float> xyz_;
};

#ifdef RS_TRACKER_HAVE_EIGEN
using Isometry3f = Eigen::Isometry3f;
inline void ToColMajor(const Isometry3f& T, float out[16]) {
  Eigen::Map<Eigen::Matrix4f>(out) = T.matrix();
}
inline void FromColMajor(const float in[16], Isometry3f* T) {
  T->matrix() = Eigen::Map<const Eigen::Matrix4f>(in);
}
#else
// 4 x 4 float, column-major (Eigen::Isometry3f::matrix() layout).
struct Isometry3f {
  std::array<float, 16> m{{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}};
  static Isometry3f Identity() { return Isometry3f{}; }
  float& operator()(int r, int c) { return m[c * 4 + r]; }
  float operator()(int r, int c) const { return m[c * 4 + r]; }
  Isometry3f operator*(const Isometry3f& o) const {
    Isometry3f out;
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) {
        float s = 0.f;
        for (int k = 0; k < 4; ++k) s += (*this)(r, k) * o(k, c);
        out(r, c) = s;
      }
    return out;
  }
};
inline void ToColMajor(const Isometry3f& T, float out[16]) {
  for (int k = 0; k < 16; ++k) out[k] = T.m[k];
}
inline void FromColMajor(const float in[16], Isometry3f* T) {
  for (int k = 0; k < 16; ++k) T->m[k] = in[k];
}
#endif

// HIP / RCCL / argument errors of the C ABI (status < 0).
class GpuError : public std::runtime_error {
 public:
  GpuError(int status, const std::string& what)
      : std::runtime_error(what + ": " + rst_status_string(status)), status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

namespace gpu {

inline int Check(int status, const char* what) {
  if (status < 0) throw GpuError(status, what);
  return status;
}

// One GPU + one HIP stream (rst_ctx).  Not copyable; one per thread that
// calls in concurrently.
class Context {
 public:
  explicit Context(int device = 0) { Check(rst_ctx_create(device, &ctx_), "rst_ctx_create"); }
  ~Context() { rst_ctx_destroy(ctx_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  rst_ctx* get() const { return ctx_; }

 private:
  rst_ctx* ctx_ = nullptr;
};

// Per-thread context on device 0 (the reference's free functions take no
// context; thread_local keeps them reentrant like the reference's).
inline Context& DefaultContext() {
  thread_local Context ctx{0};
  return ctx;
}

}  // namespace gpu
}  // namespace rs_tracker
