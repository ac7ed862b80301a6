// rs_tracker/align/align_icp.hpp -- the reference's align-module C++ API
// (yycho0108/RealsenseTracker rs_tracker/align/include/rs_tracker/align/
// align_icp.hpp:14-24), header-only, over the MI355X C ABI (rst_align.h).
//
// A caller of the reference switches by including this header instead of
// the original and linking librst_align.so.  Names, argument meaning and
// the bool contract are the reference's:
//
//   bool SolveKabsch(src, dst, indices, weights, &xfm);      // :14-17
//   bool AlignIcp3d(src, dst, dst_tree, max_iter, &xfm);      // :19-21
//   bool AlignIcp3d(src, dst, max_iter, &xfm);                // :23-24
//
// The Eigen / cho_util types are replaced by layout-identical minimal
// stand-ins (rs_tracker/common/types.hpp): Cloud3f = 3 x N column-major
// float (AoS xyz), Isometry3f = 4 x 4 column-major float.  KDTree3f becomes
// an owning handle to the device-resident target index; unlike the
// reference's tree it copies dst, so dst need not outlive it.
//
// HIP / RCCL failures (which the reference cannot have) throw
// rs_tracker::GpuError; the reference's own failure conditions return false.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "rs_tracker/common/types.hpp"

namespace rs_tracker {

// Exact 1-NN index over a target cloud (replaces KDTree3f{dst, 16},
// common/include/rs_tracker/common/kdtree.hpp:27-57).
class KDTree3f {
 public:
  KDTree3f(const Cloud3f& dst, int leaf_max_size = 16, gpu::Context& ctx = gpu::DefaultContext())
      : ctx_(&ctx) {
    (void)leaf_max_size;  // the index's leaves hold <= 16 points (kLeafTarget)
    gpu::Check(rst_target_build(ctx.get(), dst.data(), dst.cols(), &t_), "rst_target_build");
  }
  ~KDTree3f() { rst_target_free(t_); }
  KDTree3f(const KDTree3f&) = delete;
  KDTree3f& operator=(const KDTree3f&) = delete;
  KDTree3f(KDTree3f&& o) noexcept : ctx_(o.ctx_), t_(std::exchange(o.t_, nullptr)) {}

  // query(p, k, idx, d2) for k = 1 (kdtree.hpp:51-57): exact nearest
  // neighbour, squared distance.
  void query(const float* p, int num_closest, int32_t* out_indices, float* out_sq_dists) const {
    if (num_closest == 1)
      gpu::Check(rst_target_query_nn(ctx_->get(), t_, p, 1, out_indices, out_sq_dists), "query");
    else
      gpu::Check(rst_target_query_knn(ctx_->get(), t_, p, 1, num_closest, out_indices,
                                       out_sq_dists),
                 "query_knn");
  }
  // Batched form (the GPU's natural unit).
  void query_batch(const Cloud3f& q, std::vector<int32_t>* idx, std::vector<float>* d2) const {
    idx->resize(q.cols());
    d2->resize(q.cols());
    gpu::Check(rst_target_query_nn(ctx_->get(), t_, q.data(), q.cols(), idx->data(), d2->data()),
               "query_batch");
  }

  rst_target* handle() const { return t_; }
  gpu::Context& context() const { return *ctx_; }

 private:
  gpu::Context* ctx_;
  rst_target* t_ = nullptr;
};

namespace detail {
inline bool Align(gpu::Context& ctx, const Cloud3f& src, rst_target* tgt, int64_t m,
                  const int max_iter, Isometry3f* const transform) {
  // align_icp.cpp:77-79: fewer than 3 points -> false, transform untouched
  if (src.cols() < 3 || m < 3) return false;
  rst_icp_opts o;
  rst_icp_opts_default(&o);
  o.max_iter = max_iter;
  float pose[16];
  ToColMajor(*transform, pose);
  float mean_cost = 0.f;
  const int s = rst_icp_align(ctx.get(), src.data(), src.cols(), tgt, &o, pose, &mean_cost);
  gpu::Check(s, "rst_icp_align");
  FromColMajor(pose, transform);  // :156 written on both true and false
  return s == RST_OK;
}
}  // namespace detail

inline bool SolveKabsch(const Cloud3f& src, const Cloud3f& dst,
                        const std::vector<std::pair<int, int>>& indices,
                        const std::vector<float>& weights, Isometry3f* const xfm) {
  if (src.cols() < 3 || dst.cols() < 3) return false;  // align_icp.cpp:22-24
  std::vector<int32_t> pairs(2 * indices.size());
  for (size_t c = 0; c < indices.size(); ++c) {
    pairs[2 * c] = indices[c].first;
    pairs[2 * c + 1] = indices[c].second;
  }
  float pose[16];
  const int s = rst_solve_kabsch(gpu::DefaultContext().get(), src.data(), src.cols(), dst.data(),
                                 dst.cols(), pairs.data(), weights.empty() ? nullptr : weights.data(),
                                 (int64_t)indices.size(), pose);
  gpu::Check(s, "rst_solve_kabsch");
  if (s != RST_OK) return false;
  FromColMajor(pose, xfm);
  return true;
}

inline bool AlignIcp3d(const Cloud3f& src, const Cloud3f& dst, const KDTree3f& dst_tree,
                       const int max_iter, Isometry3f* const transform) {
  return detail::Align(dst_tree.context(), src, dst_tree.handle(), dst.cols(), max_iter, transform);
}

inline bool AlignIcp3d(const Cloud3f& src, const Cloud3f& dst, const int max_iter,
                       Isometry3f* const transform) {
  if (src.cols() < 3 || dst.cols() < 3) return false;  // before the tree build (:77-79)
  const KDTree3f tree{dst, 16};                          // :165
  return AlignIcp3d(src, dst, tree, max_iter, transform);
}

}  // namespace rs_tracker
