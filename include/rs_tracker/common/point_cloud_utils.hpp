// rs_tracker/common/point_cloud_utils.hpp -- the reference's cloud utilities
// that sit on the ICP path (rs_tracker/common/include/rs_tracker/common/
// point_cloud_utils.hpp:9-28), header-only over the MI355X C ABI
// (include/rst_align.h).  Same names and argument meaning; cloud_out may
// alias cloud_in, as in the reference (point_cloud_utils.cpp:50-58).
#ifndef RS_TRACKER_COMMON_POINT_CLOUD_UTILS_HPP_
#define RS_TRACKER_COMMON_POINT_CLOUD_UTILS_HPP_

#include "rs_tracker/common/types.hpp"

namespace rs_tracker {

// point_cloud_utils.cpp:34-68: the first point of every voxel
// floor(p / voxel_size), in the reference's order: its std::unordered_map's
// iteration (point_cloud_utils.cpp:54-57), replayed on the device.
inline void DownsampleVoxel(const Cloud3f& cloud_in, const float voxel_size,
                            Cloud3f* const cloud_out) {
  Cloud3f tmp(cloud_in.cols());
  int64_t n = 0;
  gpu::Check(rst_downsample_voxel(gpu::DefaultContext().get(), cloud_in.data(), cloud_in.cols(),
                                  voxel_size, tmp.data(), &n),
             "rst_downsample_voxel");
  tmp.Resize(n);
  *cloud_out = std::move(tmp);
}

// point_cloud_utils.cpp:163-174: drop points with a non-finite coordinate.
inline void RemoveNans(const Cloud3f& cloud_in, Cloud3f* const cloud_out) {
  Cloud3f tmp(cloud_in.cols());
  int64_t n = 0;
  gpu::Check(rst_remove_nans(gpu::DefaultContext().get(), cloud_in.data(), cloud_in.cols(),
                             tmp.data(), &n),
             "rst_remove_nans");
  tmp.Resize(n);
  *cloud_out = std::move(tmp);
}

// point_cloud_utils.cpp:92-98 (fp64 accumulation on the device).
inline void ComputeCentroid(const Cloud3f& cloud, float centroid[3]) {
  gpu::Check(rst_compute_centroid(gpu::DefaultContext().get(), cloud.data(), cloud.cols(),
                                  centroid),
             "rst_compute_centroid");
}

}  // namespace rs_tracker

#endif  // RS_TRACKER_COMMON_POINT_CLOUD_UTILS_HPP_
