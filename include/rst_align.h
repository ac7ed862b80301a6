/*
 * rst_align.h -- C ABI of the MI355X-native rs_tracker/align ICP path.
 *
 * Drop-in boundary for the reference's align module
 * (yycho0108/RealsenseTracker, rs_tracker/align/include/rs_tracker/align/
 * align_icp.hpp:14-24).  Plain pointers and sizes only; every entry point
 * returns an int status:
 *     0  ok
 *     1  the reference's `false` (fewer than 3 points, or mean cost NaN /
 *        >= 10000 -- align_icp.cpp:77-79,157-160)
 *    <0  rst_status error (HIP / RCCL / argument)
 *
 * Clouds are AoS xyz float32 (point i at xyz[3i..3i+2]); this is the byte
 * layout of the reference's Cloud3f = cho::core::PointCloud<float,3>
 * (Eigen 3xN column-major, types.hpp:14).  Poses are 4x4 float32
 * column-major, the layout of Eigen::Isometry3f::matrix().
 *
 * Entry points ending in _device take device (HBM) pointers; the others take
 * host pointers and copy through pinned staging buffers owned by the context.
 * A context is bound to one GPU and one HIP stream; calls on one context are
 * not thread-safe, distinct contexts are independent (reentrant).
 */
#ifndef RST_ALIGN_H_
#define RST_ALIGN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RST_ABI_VERSION 1

typedef enum {
  RST_OK = 0,
  RST_FALSE = 1,          /* reference bool false */
  RST_E_ARG = -1,         /* invalid argument */
  RST_E_HIP = -2,         /* HIP runtime error */
  RST_E_NOMEM = -3,       /* allocation failure */
  RST_E_NODEVICE = -4,    /* no GPU / bad device ordinal */
  RST_E_COMM = -5,        /* RCCL error */
  RST_E_STATE = -6        /* object in wrong state (e.g. normals missing) */
} rst_status;

typedef enum {
  /* the reference's point-to-point ICP with annealed Geman-McClure weights,
   * fp64 cross-covariance, Kabsch/SVD, fixed max_iter (align_icp.cpp:92-153) */
  RST_P2POINT_REF = 0,
  /* build's own point-to-plane Gauss-Newton (no reference counterpart;
   * needs target normals; converges on |dxi| < eps) */
  RST_P2PLANE = 1
} rst_icp_mode;

typedef enum {
  /* the reference's own rounding (align_icp.cpp:101,113,120-122 and
   * point_cloud_utils.cpp:92-98): the source centroid, dst_mean and cost are
   * float32 sums taken sequentially in ascending source index, exactly as
   * the CPU loop rounds them; the covariance is the fp64 sum of the same
   * float products.  Bit-identical means and cost; the default. */
  RST_SUM_REF = 0,
  /* fp64 partial sums in any order (one pass, no sequential step): the
   * throughput mode.  Differs from the reference by the loop's own
   * fp32-vs-fp64 sensitivity: NOT within a 1e-4 pose gate of it -- up to
   * ~1e-3 m / 2e-4 rad after 128 iterations on 640x480 frame pairs
   * (tests/golden/fp64_gate.json). */
  RST_SUM_FP64 = 1
} rst_sum_mode;

typedef struct {
  int32_t max_iter;       /* 128 at both reference call sites */
  int32_t mode;           /* rst_icp_mode */
  float mu0;              /* initial mu (align_icp.cpp:91): 1.0 */
  int32_t anneal_every;   /* mu /= anneal_div every N iters (:96-98): 8 */
  float anneal_div;       /* 1.4 */
  float p2plane_eps;      /* P2PLANE: stop when |xi| < eps (1e-6) */
  float p2plane_mu;       /* P2PLANE: GM scale on plane residual (m^2) */
  float p2plane_max_dist; /* P2PLANE: reject NN beyond this (m); 0 = off */
  int32_t sum_mode;       /* rst_sum_mode (P2POINT_REF only; sharded, the
                           * RST_SUM_REF chains are relayed rank to rank:
                           * every rank gets the same bit-exact sums) */
  int32_t n_total;        /* sharded align: the points of ALL shards when the
                           * caller knows them (> 0: no count all-reduce and no
                           * host round trip before the loop; must equal the
                           * sum of n_shard over the ranks); 0 = all-reduce the
                           * count (one host synchronisation per align) */
  int32_t reserved[6];
} rst_icp_opts;

typedef struct {
  float fx, fy, cx, cy;   /* pinhole intrinsics (rs_driver.cpp:264-280) */
  int32_t width, height;
  float depth_scale;      /* metres per depth unit (RealSense: 0.001) */
  float min_depth, max_depth; /* valid range in metres; 0 = no limit */
} rst_intrinsics;

typedef struct rst_ctx rst_ctx;
typedef struct rst_target rst_target;
typedef struct rst_scene rst_scene;
typedef struct rst_comm rst_comm;

/* ---- library ------------------------------------------------------------ */
int rst_abi_version(void);
const char* rst_status_string(int status);
void rst_icp_opts_default(rst_icp_opts* opts);
int rst_device_count(int* count);

/* ---- context (one GPU, one stream) -------------------------------------- */
int rst_ctx_create(int device, rst_ctx** out);
int rst_ctx_destroy(rst_ctx* ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream()); NULL
 * restores the context's own stream. */
int rst_ctx_set_stream(rst_ctx* ctx, void* hip_stream);
int rst_ctx_synchronize(rst_ctx* ctx);
/* Average duration (ms) of the dominant per-iteration kernel over the last
 * align call, measured with HIP events on the context's stream; and the
 * number of launches it covers.  Used by bench.py's roofline. */
int rst_ctx_last_kernel_time(rst_ctx* ctx, float* avg_ms, int32_t* launches);
/* The same events split over the whole iteration: avg_ms[0] = kernel 1
 * (k_icp_nn, the certificate stream), [1] = kernel 2 (k_icp_fb, the
 * searches), [2] = the rest (reductions and the solve; RST_SUM_REF: also the
 * sequential sums). */
int rst_ctx_last_iteration_times(rst_ctx* ctx, float avg_ms[3], int32_t* iterations);
/* Iterations run by the last align finished on this context (the entry
 * points without an iterations_run output: the sharded aligns). */
int rst_ctx_last_iterations(rst_ctx* ctx, int32_t* iterations);
/* hipGraph mode (BASELINE configs[4]): each align's iteration loop is
 * captured and replayed as one graph (the executable for a given iteration
 * count and mode is kept on the context and updated in place with the next
 * align's arguments).  Same results; not used by the sharded (RCCL) align or
 * while kernel timing is on.  0 = off (default). */
int rst_ctx_enable_graphs(rst_ctx* ctx, int enable);
/* Per-iteration kernel timing (HIP events around the dominant kernel on the
 * context's stream): 0 = off (default), 1 = every iteration, k > 1 = every
 * k-th iteration (fewer events in a timed loop). */
int rst_ctx_enable_kernel_timing(rst_ctx* ctx, int enable);

/* ---- device buffers ------------------------------------------------------ */
/* Plain HBM allocations on the context's device, for callers that hand the
 * *_device entry points their own buffers (bindings, tests, the bench)
 * without a second runtime (e.g. torch's) in the process.  Copies are
 * ordered on the context's stream and complete before returning. */
int rst_dev_alloc(rst_ctx* ctx, int64_t bytes, void** d_out);
int rst_dev_free(rst_ctx* ctx, void* d);
int rst_dev_upload(rst_ctx* ctx, void* d_dst, const void* h_src, int64_t bytes);
int rst_dev_download(rst_ctx* ctx, void* h_dst, const void* d_src, int64_t bytes);

/* ---- target index (replaces KDTree3f{dst,16}; kdtree.hpp:27-57) --------- */
/* Builds the exact-NN index (Morton-ordered bounding-volume hierarchy) over
 * m target points.  Unlike the reference's tree the handle owns a device
 * copy, so dst need not outlive it. */
int rst_target_build(rst_ctx* ctx, const float* xyz, int64_t m,
                     rst_target** out);
int rst_target_build_device(rst_ctx* ctx, const float* d_xyz, int64_t m,
                            rst_target** out);
int rst_target_free(rst_target* tgt);
int64_t rst_target_size(const rst_target* tgt);

/* kNN-PCA normals (ComputeNormals + OrientNormals,
 * point_cloud_utils.cpp:176-216), stored in the handle for P2PLANE. */
int rst_target_compute_normals(rst_ctx* ctx, rst_target* tgt, int k,
                               const float viewpoint[3]);
/* Image-grid normals (point-to-plane perf mode; no reference counterpart):
 * for a target prepared from a depth frame (rst_frame_prepare_device / the
 * pyramid), the PCA normal of each point's (2 radius + 1)^2 pixel window
 * (radius 1 or 2; window points farther than 5 pixel pitches excluded),
 * oriented as OrientNormals.  The kNN-PCA normals above stay the reference
 * semantics.  RST_E_STATE for a target without a pixel grid. */
int rst_target_compute_grid_normals(rst_ctx* ctx, rst_target* tgt, int radius,
                                    const float viewpoint[3]);
/* Copy normals out in the target's original point order (host m*3). */
int rst_target_get_normals(rst_ctx* ctx, const rst_target* tgt,
                           float* normals);

/* Exact 1-NN per query (KDTree3f::query(p, 1, &j, &d2), kdtree.hpp:51-57):
 * idx = target index, d2 = squared L2 distance in float with nanoflann's
 * op order; ties -> lowest index; non-finite query -> (0, FLT_MAX). */
int rst_target_query_nn(rst_ctx* ctx, const rst_target* tgt, const float* q,
                        int64_t nq, int32_t* idx, float* d2);
int rst_target_query_nn_device(rst_ctx* ctx, const rst_target* tgt,
                               const float* d_q, int64_t nq, int32_t* d_idx,
                               float* d_d2);
/* The same exact 1-NN, for spatially coherent query batches (e.g. one
 * frame's points in scan order) with optional warm candidates: warm[i] =
 * a target index believed close to q[i] (the previous frame's answer), <0
 * = none; warm may be NULL.  Runs the ICP loop's wave-cooperative search;
 * results are identical to rst_target_query_nn for any input. */
int rst_target_query_nn_warm(rst_ctx* ctx, const rst_target* tgt, const float* q,
                             int64_t nq, const int32_t* warm, int32_t* idx,
                             float* d2);
/* Exact k-NN (k <= 32), results sorted by (d2, idx). */
int rst_target_query_knn(rst_ctx* ctx, const rst_target* tgt, const float* q,
                         int64_t nq, int k, int32_t* idx, float* d2);

/* ---- ICP (AlignIcp3d, align_icp.cpp:73-167) ----------------------------- */
/* 5-arg overload: prebuilt target.  pose_inout = initial guess in, result
 * out (left untouched on the early false return).  mean_cost may be NULL;
 * for RST_P2POINT_REF it is sqrt(sum d2 / n) of the last iteration (:157). */
int rst_icp_align(rst_ctx* ctx, const float* src, int64_t n,
                  const rst_target* tgt, const rst_icp_opts* opts,
                  float pose_inout[16], float* mean_cost);
/* 4-arg overload: builds the target index from dst first (:163-167). */
int rst_icp_align_clouds(rst_ctx* ctx, const float* src, int64_t n,
                         const float* dst, int64_t m,
                         const rst_icp_opts* opts, float pose_inout[16],
                         float* mean_cost);
/* Device-resident source (HBM pointer); pose stays a host array. */
int rst_icp_align_device(rst_ctx* ctx, const float* d_src, int64_t n,
                         const rst_target* tgt, const rst_icp_opts* opts,
                         float pose_inout[16], float* mean_cost);
/* Source already prepared as a target handle (its Morton order is reused
 * as a coherent query order -- the replay loop uses each frame twice). */
int rst_icp_align_prepared(rst_ctx* ctx, const rst_target* src,
                           const rst_target* tgt, const rst_icp_opts* opts,
                           float pose_inout[16], float* mean_cost,
                           int32_t* iterations_run);

/* rst_icp_align_prepared split in two, so several frame pairs can be in
 * flight on one GPU (one context -- one HIP stream -- each): _async enqueues
 * the whole loop and returns RST_OK, or RST_FALSE for the reference's early
 * false (nothing enqueued), or an error; _wait blocks until that align is
 * done and returns what rst_icp_align_prepared would (pose_inout in: the
 * same initial guess given to _async; out: the result).  One align per
 * context at a time (RST_E_STATE otherwise).  src and tgt must stay alive
 * until _wait returns. */
int rst_icp_align_prepared_async(rst_ctx* ctx, const rst_target* src,
                                 const rst_target* tgt, const rst_icp_opts* opts,
                                 const float pose_in[16]);
int rst_icp_align_wait(rst_ctx* ctx, float pose_inout[16], float* mean_cost,
                       int32_t* iterations_run);

/* A batch of nb independent frame pairs aligned in lockstep on one context:
 * AlignIcp3d(src[p], tgt[p]) from pose_in[16 p .. 16 p + 16) for every p,
 * each result bit-identical to aligning the pair alone, but one launch of
 * each loop kernel covers the whole batch (the GPU runs only a few kernels
 * of independent streams at once; a batch hands it nb pairs' work per
 * launch).  Pairs with the reference's early false (< 3 points; < 6 for
 * RST_P2PLANE) are left out and report it.  One align or batch in flight
 * per context (RST_E_STATE otherwise); the targets must stay alive until
 * _wait.  _wait: poses_inout (nb x 16), mean_costs (nb, may be NULL),
 * status (nb: RST_OK / RST_FALSE per pair), iterations (nb, may be NULL);
 * returns RST_OK or the first error. */
int rst_icp_align_batch_async(rst_ctx* ctx, int32_t nb, const rst_target* const* src,
                              const rst_target* const* tgt, const rst_icp_opts* opts,
                              const float* poses_in);
int rst_icp_align_batch_wait(rst_ctx* ctx, float* poses_inout, float* mean_costs,
                             int32_t* status, int32_t* iterations);

/* Coarse-to-fine ICP over pyramid levels (BASELINE configs[4]; the
 * reference has no pyramid): level 0 is the finest, nlevels-1 the coarsest.
 * Runs levels nlevels-1 .. 0, iters[l] iterations each, every level starting
 * from the previous level's pose -- chained on the device, so the whole
 * pyramid is enqueued at once.  Equivalent to calling
 * rst_icp_align_prepared(src[l], tgt[l], opts{max_iter = iters[l]}, pose)
 * coarsest first with one pose array (a level whose early false leaves the
 * pose untouched is skipped the same way).  RST_FALSE, nothing enqueued,
 * when level 0 has < 3 source or target points (< 6 source points for
 * RST_P2PLANE); _wait then reports it too.  Finish with rst_icp_align_wait
 * (level 0's result; iterations_run = level 0's). */
int rst_icp_align_pyramid_async(rst_ctx* ctx, const rst_target* const* src,
                                const rst_target* const* tgt, int nlevels,
                                const int32_t* iters, const rst_icp_opts* opts,
                                const float pose_in[16]);

/* The per-iteration solve of AlignIcp3d / SolveKabsch (align_icp.cpp:58-69,
 * 139-151) run by the device solve kernel on a given fp64 cross-covariance
 * (column-major) and float means: R = float(U V^T), R.col(2) *= -1 when
 * det(R) < 0, t = dmean - R smean, quaternion round trip. */
int rst_kabsch_solve(rst_ctx* ctx, const double cov[9], const float smean[3],
                     const float dmean[3], float pose_out[16]);

/* SolveKabsch (align_icp.cpp:18-71, declared align_icp.hpp:14-17): weighted
 * Kabsch over k correspondences pairs[2c] = src index, pairs[2c+1] = dst
 * index; weights may be NULL (unweighted branch, :38-45).  Means and the
 * fp64 covariance are computed on the device, then the same solve as
 * rst_kabsch_solve.  RST_FALSE when n < 3 or m < 3 (pose untouched, :22-24);
 * k == 0 gives what the reference computes from its 0/0 means: RST_OK,
 * R = I, t = NaN.  RST_E_ARG for an index out of range. */
int rst_solve_kabsch(rst_ctx* ctx, const float* src, int64_t n,
                     const float* dst, int64_t m, const int32_t* pairs,
                     const float* weights, int64_t k, float pose_out[16]);

/* ComputeCentroid (point_cloud_utils.cpp:92-98): the reference's fp32
 * sequential sum in input order times float(1.0 / n), bit-exact. */
int rst_compute_centroid(rst_ctx* ctx, const float* xyz, int64_t n,
                         float out[3]);

/* ---- depth -> xyz (rs2::pointcloud::calculate at data_source_rs.cpp:89) -- */
/* Pinhole deprojection of a u16 depth image.  Invalid pixels (0, or outside
 * [min_depth,max_depth]) are dropped when keep_invalid == 0 (order
 * preserving compaction) or written as (0,0,0) like the reference's NaN->0
 * copy (data_source_rs.cpp:34-41).  n_out receives the point count. */
int rst_unproject(rst_ctx* ctx, const uint16_t* depth,
                  const rst_intrinsics* K, int keep_invalid, float* xyz_out,
                  int64_t* n_out);
int rst_unproject_device(rst_ctx* ctx, const uint16_t* d_depth,
                         const rst_intrinsics* K, int keep_invalid,
                         float* d_xyz_out, int64_t* n_out);
/* Fused frame preparation: depth (device) -> points -> target handle
 * (+ normals: normals_k > 0 kNN-PCA with k = normals_k, normals_k = -1 / -2
 * image-grid normals of radius 1 / 2, 0 none; viewpoint = the camera).
 * One call per incoming frame. */
int rst_frame_prepare_device(rst_ctx* ctx, const uint16_t* d_depth,
                             const rst_intrinsics* K, int normals_k,
                             rst_target** out);
/* Decimated deprojection (coarse-to-fine pyramid, BASELINE configs[4]; no
 * reference counterpart): every stride-th pixel of every stride-th row,
 * i.e. pixel (stride*ul, stride*vl) deprojected with the full image's
 * intrinsics K, so the points are exactly the level-0 points of those
 * pixels.  stride 1 = rst_unproject_device. */
int rst_unproject_strided_device(rst_ctx* ctx, const uint16_t* d_depth,
                                 const rst_intrinsics* K, int stride,
                                 int keep_invalid, float* d_xyz_out,
                                 int64_t* n_out);
/* rst_frame_prepare_device for levels 0..nlevels-1 (stride 2^l) of one
 * depth frame: out_levels[l] receives level l's target handle (all freed
 * and NULL on error). */
int rst_frame_prepare_pyramid_device(rst_ctx* ctx, const uint16_t* d_depth,
                                     const rst_intrinsics* K, int nlevels,
                                     int normals_k, rst_target** out_levels);

/* ---- cloud preprocessing the callers run before AlignIcp3d -------------- */
/* RemoveNans (point_cloud_utils.cpp:163-174): keep the points whose three
 * coordinates are finite, in input order.  out holds >= n points; n_out
 * receives the count.  Returns RST_OK. */
int rst_remove_nans(rst_ctx* ctx, const float* xyz, int64_t n, float* out,
                    int64_t* n_out);
int rst_remove_nans_device(rst_ctx* ctx, const float* d_xyz, int64_t n,
                           float* d_out, int64_t* n_out);
/* DownsampleVoxel (point_cloud_utils.cpp:34-68): the first point (lowest
 * input index) of every voxel (int)floor(p / voxel_size), emitted in the
 * reference's order: the iteration order of its std::unordered_map (:54-57),
 * libstdc++'s container with the classic boost::hash_combine (Boost <= 1.80)
 * replayed on the device (voxel.hip).  NaN / out-of-int-range
 * coordinates key to INT_MIN as the reference's float->int cast does on
 * x86-64.  voxel_size must be > 0 and n < 2^30 (RST_E_ARG otherwise);
 * out holds >= n points. */
int rst_downsample_voxel(rst_ctx* ctx, const float* xyz, int64_t n,
                         float voxel_size, float* out, int64_t* n_out);
int rst_downsample_voxel_device(rst_ctx* ctx, const float* d_xyz, int64_t n,
                                float voxel_size, float* d_out,
                                int64_t* n_out);

/* ---- FPFH global initialisation ------------------ */
/* ComputeFpfh(cloud, viewpoint, normal_k, feature_radius, &fpfh)
 * (fpfh.cpp:248-262): index, kNN-PCA normals oriented to the viewpoint
 * (normal_k in {8, 16, 32}, n >= normal_k), SPFH over the radius neighbours
 * (|p - q|^2 < r^2), FPFH = sum over neighbours but self of spfh / dist,
 * each 11-bin histogram normalised (fpfh.cpp:114-165).  fpfh_out: n x 33
 * floats, input order. */
int rst_compute_fpfh(rst_ctx* ctx, const float* xyz, int64_t n,
                     const float viewpoint[3], int normal_k, float radius,
                     float* fpfh_out);
/* ComputeMatches(src, dst, k) (fpfh.cpp:285-300): the exact k (1 or 2)
 * nearest dst features of every src feature (33-D, nanoflann metric_L2
 * arithmetic, ties to the lower index); idx_out n x k, d2_out (optional)
 * n x k. */
int rst_compute_matches(rst_ctx* ctx, const float* src_feat, int64_t n,
                        const float* dst_feat, int64_t m, int k,
                        int32_t* idx_out, float* d2_out);

/* ---- CloudAccumulator (rs_replay_app.cpp:76-129) -- */
/* A voxel map on the device: AddCloud(xfm, cloud) inserts xfm * p for
 * every point whose voxel (int)(p * inv) -- inv = float(1.0 / voxel_size),
 * truncation, NaN / out-of-range -> INT_MIN -- is new; the first point added
 * to a voxel stays.  Extract returns the points in the reference's order,
 * its std::unordered_map's iteration (rs_replay_app.cpp:112-121; as
 * rst_downsample_voxel). */
typedef struct rst_accum rst_accum;
int rst_accum_create(rst_ctx* ctx, float voxel_size, rst_accum** out);
int rst_accum_destroy(rst_accum* a);
int rst_accum_add(rst_accum* a, const float pose[16], const float* xyz, int64_t n);
int rst_accum_add_device(rst_accum* a, const float pose[16], const float* d_xyz,
                         int64_t n);
int rst_accum_size(const rst_accum* a, int64_t* n);
/* out holds >= size points */
int rst_accum_extract(rst_accum* a, float* out, int64_t* n_out);

/* ---- GICP, the align module's second path -------- */
/* ComputeCovariances(tree, cloud, covs, use_gicp) (point_cloud_utils.cpp:
 * 100-161) on a prepared cloud: per point the 32 nearest others (33-NN,
 * self first), fp32 centroid and sum of outer products / 31; use_gicp:
 * U diag(1, 1, 1e-2) U^T.  covs_out: m x 9 floats (3x3 column-major, as
 * Eigen::Matrix3f), original point order. */
int rst_compute_covariances(rst_ctx* ctx, const rst_target* tgt, int use_gicp,
                            float* covs_out);
/* ComputeAlignment(src, dst, src_covs, dst_covs, dst_indices, seed, &T)
 * (align_gicp.cpp:41-103): minimises 1/2 sum Huber_0.5(|C_i^-1/2 (R s_i +
 * t - d_j)|^2), C_i = S_d + R S_s R^T (gicp_cost.hpp:40-73), from seed, by
 * Levenberg-Marquardt (fp64, at most max_iter cost evaluations; the Ceres
 * solver it replaces is not reproduced step by step, only its objective).
 * pose_out col-major 4x4; cost_out = the final cost (Ceres final_cost);
 * RST_FALSE when the pose is not finite. */
int rst_gicp_solve(rst_ctx* ctx, const float* src, int64_t n, const float* dst,
                   int64_t m, const float* src_covs, const float* dst_covs,
                   const int32_t* dst_idx, const float seed[16], int max_iter,
                   float pose_out[16], double* cost_out, int32_t* iters_out);
/* ComputeAlignment(src, dst, &T) (align_gicp.cpp:105-163): covariances of
 * both clouds (k = 32, use_gicp = false), estimate = Identity (the
 * reference ignores T's value), outer_iters (reference: 16) x {exact 1-NN
 * of estimate * src in dst; the solve above seeded at estimate}.
 * RST_FALSE (cost = inf) when the result is not finite (:145-150). */
int rst_gicp_align(rst_ctx* ctx, const float* src, int64_t n, const float* dst,
                   int64_t m, int outer_iters, int max_inner, float pose_out[16],
                   double* cost_out);

/* ---- synthetic frame source (driver; replaces the camera) --------------- */
/* Procedural room (walls + random spheres/boxes), seeded. */
int rst_scene_create(uint64_t seed, rst_scene** out);
int rst_scene_destroy(rst_scene* scene);
/* Ray-cast u16 depth for camera pose T_wc (camera->world, col-major 4x4):
 * z-depth quantised by depth_scale, Gaussian noise sigma (metres), a
 * fraction of pixels dropped to 0; deterministic in noise_seed. */
int rst_scene_render_depth(const rst_scene* scene, const float T_wc[16],
                           const rst_intrinsics* K, uint64_t noise_seed,
                           float noise_sigma, float invalid_frac,
                           uint16_t* depth_out);
/* Smooth camera trajectory through the room; frame -> T_wc. */
int rst_scene_trajectory(const rst_scene* scene, int32_t frame,
                         float T_wc_out[16]);
/* RandomSource::GetCloud (data_source.hpp:29-36): uniform [-1,1]^3,
 * seeded (the reference's is unseeded). */
int rst_random_cloud(uint64_t seed, int64_t n, float* xyz_out);

/* ---- multi-GPU: source shards + one RCCL all-reduce per iteration ------- */
#define RST_COMM_ID_BYTES 128
int rst_comm_get_unique_id(char id_out[RST_COMM_ID_BYTES]);
int rst_comm_create(rst_ctx* ctx, const char id[RST_COMM_ID_BYTES],
                    int nranks, int rank, rst_comm** out);
int rst_comm_destroy(rst_comm* comm);
/* Every rank passes its own source shard -- rank r the r-th contiguous
 * stretch of the source's order -- and the full (replicated) target; every
 * rank solves the same pose.  Per iteration: RST_SUM_FP64 one all-reduce of
 * 16 fp64 partial sums, RST_P2PLANE one of the 30-double 6x6 / 6x1 normal
 * equations, RST_SUM_REF the sequential sums' relay (an all-gather of 32 B
 * per rank, a 16 B hop per rank, a 16 B broadcast) and one all-reduce of the
 * 9 covariance sums.  n_total = sum of shard sizes (ranks agree). */
int rst_icp_align_sharded_device(rst_ctx* ctx, rst_comm* comm,
                                 const float* d_src_shard, int64_t n_shard,
                                 const rst_target* tgt,
                                 const rst_icp_opts* opts,
                                 float pose_inout[16], float* mean_cost);
/* The same with a source shard prepared once (rst_target_build_device or
 * rst_frame_prepare_device, with or without an index): no per-call Morton
 * sort of the shard.  With opts->n_total set, the call enqueues the whole
 * loop (RCCL all-reduces included) and synchronises only to read the pose. */
int rst_icp_align_sharded_prepared(rst_ctx* ctx, rst_comm* comm, const rst_target* src_shard,
                                   const rst_target* tgt, const rst_icp_opts* opts,
                                   float pose_inout[16], float* mean_cost);

#ifdef __cplusplus
}
#endif
#endif /* RST_ALIGN_H_ */
