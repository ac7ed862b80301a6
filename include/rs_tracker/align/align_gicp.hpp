// rs_tracker/align/align_gicp.hpp -- the reference's GICP entry points
// (rs_tracker/align/include/rs_tracker/align/align_gicp.hpp:15-27) and the
// helpers it uses (point_cloud_utils.hpp:12-20), header-only over the
// MI355X C ABI (rst_align.h).  Covariances travel as 3 x 3 column-major
// float (Eigen::Matrix3f's layout): Matrix3f below.
//
//   float ComputeAlignment(src, dst, &T);                       // :23-24
//   float ComputeAlignment(src, dst, src_covs, dst_covs,
//                          dst_indices, seed, &T);               // :15-21
//   void ComputeCovariances(tree, cloud, &covs, use_gicp);
//   void FindCorrespondences(tree, source, &indices, &sq_dists);
//
// The three-argument form starts from Identity whatever T holds, as the
// reference does (align_gicp.cpp:127-129).  A non-finite result returns
// +inf and leaves T untouched.
#pragma once

#include <array>
#include <cstdint>
#include <limits>
#include <vector>

#include "rs_tracker/align/align_icp.hpp"

namespace rs_tracker {

using Matrix3f = std::array<float, 9>;  // column-major (Eigen::Matrix3f layout)

inline void ComputeCovariances(const KDTree3f& tree, const Cloud3f& cloud,
                               std::vector<Matrix3f>* const covs, const bool use_gicp) {
  covs->resize(cloud.cols());
  gpu::Check(rst_compute_covariances(gpu::DefaultContext().get(), tree.handle(), use_gicp ? 1 : 0,
                                     covs->empty() ? nullptr : covs->front().data()),
             "rst_compute_covariances");
}

inline void FindCorrespondences(const KDTree3f& tree, const Cloud3f& source,
                                std::vector<int>* const indices,
                                std::vector<float>* const squared_distances) {
  std::vector<int32_t> idx;
  tree.query_batch(source, &idx, squared_distances);
  indices->assign(idx.begin(), idx.end());
}

inline float ComputeAlignment(const Cloud3f& src, const Cloud3f& dst,
                              const std::vector<Matrix3f>& src_covs,
                              const std::vector<Matrix3f>& dst_covs,
                              const std::vector<int>& dst_indices, const Isometry3f& seed,
                              Isometry3f* const transform, int max_iter = 64) {
  if (src.cols() < 1 || dst.cols() < 1 || (int64_t)src_covs.size() != src.cols() ||
      (int64_t)dst_covs.size() != dst.cols() || (int64_t)dst_indices.size() != src.cols())
    return std::numeric_limits<float>::infinity();
  float sd[16], out[16];
  ToColMajor(seed, sd);
  std::vector<int32_t> idx(dst_indices.begin(), dst_indices.end());
  double cost = 0.0;
  int32_t iters = 0;
  const int s = gpu::Check(
      rst_gicp_solve(gpu::DefaultContext().get(), src.data(), src.cols(), dst.data(), dst.cols(),
                     src_covs.front().data(), dst_covs.front().data(), idx.data(), sd, max_iter,
                     out, &cost, &iters),
      "rst_gicp_solve");
  if (s != RST_OK) return std::numeric_limits<float>::infinity();
  FromColMajor(out, transform);
  return (float)cost;
}

inline float ComputeAlignment(const Cloud3f& src, const Cloud3f& dst,
                              Isometry3f* const transform) {
  if (src.cols() < 1 || dst.cols() < 1) return std::numeric_limits<float>::infinity();
  float out[16];
  double cost = 0.0;
  const int s = gpu::Check(rst_gicp_align(gpu::DefaultContext().get(), src.data(), src.cols(),
                                          dst.data(), dst.cols(), 16, 64, out, &cost),
                           "rst_gicp_align");
  if (s != RST_OK) return std::numeric_limits<float>::infinity();
  FromColMajor(out, transform);
  return (float)cost;
}

}  // namespace rs_tracker
