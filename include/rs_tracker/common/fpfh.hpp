// rs_tracker/common/fpfh.hpp -- the FPFH entry points the align app uses
// (rs_tracker/common/include/rs_tracker/common/fpfh.hpp; fpfh.cpp:248-300),
// header-only over the MI355X C ABI.  Cloud33f = 33 x N column-major float
// (one feature per point), as the reference's cho_util PointCloud<float, 33>.
#pragma once

#include <cstdint>
#include <vector>

#include "rs_tracker/common/types.hpp"

namespace rs_tracker {

class Cloud33f {
 public:
  Cloud33f() = default;
  explicit Cloud33f(int64_t n) : f_(33 * n, 0.f) {}
  int64_t cols() const { return (int64_t)f_.size() / 33; }
  int64_t GetNumPoints() const { return cols(); }
  float* data() { return f_.data(); }
  const float* data() const { return f_.data(); }
  const float* GetPoint(int64_t i) const { return f_.data() + 33 * i; }

 private:
  std::vector<float> f_;
};

// ComputeFpfh(cloud, viewpoint, normal_k, feature_radius, &fpfh) (:248-262)
inline void ComputeFpfh(const Cloud3f& cloud, const float viewpoint[3], const int normal_k,
                        const float feature_radius, Cloud33f* const fpfh_out) {
  Cloud33f out(cloud.cols());
  gpu::Check(rst_compute_fpfh(gpu::DefaultContext().get(), cloud.data(), cloud.cols(), viewpoint,
                              normal_k, feature_radius, out.data()),
             "rst_compute_fpfh");
  *fpfh_out = std::move(out);
}

// ComputeMatches(src, dst, num_matches, &matches) (:285-300): row i holds
// the num_matches (1 or 2) nearest dst features of src feature i
inline void ComputeMatches(const Cloud33f& src, const Cloud33f& dst, const int num_matches,
                           std::vector<int32_t>* const matches) {
  matches->assign((size_t)src.cols() * num_matches, 0);
  gpu::Check(rst_compute_matches(gpu::DefaultContext().get(), src.data(), src.cols(), dst.data(),
                                 dst.cols(), num_matches, matches->data(), nullptr),
             "rst_compute_matches");
}

}  // namespace rs_tracker
