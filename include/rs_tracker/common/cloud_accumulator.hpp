// rs_tracker/common/cloud_accumulator.hpp -- the replay app's voxel map
// (rs_replay_app.cpp:76-129: AddCloud, GetVoxelIndex, ExtractPointCloud) on
// the device, header-only over the C ABI (rst_accum_*).  Same voxel rule
// ((xfm * p) * (1 / voxel), truncated; the first point of a voxel stays);
// ExtractPointCloud returns the points in the reference's std::unordered_map
// iteration order (rs_replay_app.cpp:112-121).
#pragma once

#include "rs_tracker/common/types.hpp"

namespace rs_tracker {

class CloudAccumulator {
 public:
  explicit CloudAccumulator(const float voxel_size = 0.05f,
                            gpu::Context& ctx = gpu::DefaultContext()) {
    gpu::Check(rst_accum_create(ctx.get(), voxel_size, &a_), "rst_accum_create");
  }
  ~CloudAccumulator() { rst_accum_destroy(a_); }
  CloudAccumulator(const CloudAccumulator&) = delete;
  CloudAccumulator& operator=(const CloudAccumulator&) = delete;

  void AddCloud(const Isometry3f& xfm, const Cloud3f& cloud) {
    float T[16];
    ToColMajor(xfm, T);
    gpu::Check(rst_accum_add(a_, T, cloud.data(), cloud.cols()), "rst_accum_add");
  }

  Cloud3f ExtractPointCloud() const {
    int64_t n = 0;
    gpu::Check(rst_accum_size(a_, &n), "rst_accum_size");
    Cloud3f out(n);
    gpu::Check(rst_accum_extract(a_, out.data(), &n), "rst_accum_extract");
    return out;
  }

 private:
  rst_accum* a_ = nullptr;
};

}  // namespace rs_tracker
