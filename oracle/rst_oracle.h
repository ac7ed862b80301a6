/*
 * rst_oracle.h -- CPU ORACLE for the rs_tracker/align ICP path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference's
 * algorithm (yycho0108/RealsenseTracker), used as the checker for the HIP
 * product path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  It is never linked into, called by, or used
 * as a fallback for realsensetracker_amd/ (the product must fail loudly when
 * its HIP library is missing).
 *
 * Parity status: the reference cannot be compiled here (Eigen, nanoflann,
 * cho_util, fmt, librealsense absent; see DESIGN.md "Oracle").  This oracle is
 * pinned against an independent numpy/scipy restatement (tests/np_restate.py)
 * and against ground-truth SE(3) on synthetic pairs; against the reference
 * binary itself it is "parity unpinned".
 *
 * Conventions
 *   clouds   : AoS xyz float32, point i at xyz[3*i .. 3*i+2]  (cho_util
 *              PointCloud<float,3> = Eigen 3xN column-major, same bytes)
 *   poses    : 4x4 float32 column-major (Eigen Isometry3f::matrix() layout),
 *              m[c*4 + r]; linear part R(r,c) = m[c*4+r], t_r = m[12+r].
 *   NN ties  : equal squared distance -> lowest target index wins
 *              (nanoflann resolves ties by traversal order; documented
 *              deviation).
 */
#ifndef RST_ORACLE_H_
#define RST_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- common/kd-tree (kdtree.hpp:27-57, nanoflann KDTreeSingleIndexAdaptor) */
typedef struct orc_kdtree orc_kdtree;

/* Build a kd-tree over m AoS points with nanoflann's middle-split rule
 * (leaf_max_size 16 at align_icp.cpp:165).  The cloud must outlive the tree
 * (kdtree.hpp:30 keeps a reference). */
orc_kdtree* orc_kdtree_build(const float* xyz, int64_t m, int leaf_max_size);
void orc_kdtree_free(orc_kdtree* t);

/* Exact k-NN of one query (kdtree.hpp:51-57, KNNResultSet, eps = 0).
 * Results sorted ascending by (d2, idx).  Slots that cannot be filled keep
 * idx = 0 / d2 = FLT_MAX, as the reference's out-params do
 * (align_icp.cpp:110-112 + KNNResultSet::init). */
void orc_kdtree_knn(const orc_kdtree* t, const float q[3], int k,
                    int32_t* idx, float* d2);

/* Batched exact 1-NN. */
void orc_nn_batch(const orc_kdtree* t, const float* q, int64_t nq,
                  int32_t* idx, float* d2);

/* Brute-force exact 1-NN (same distance arithmetic and tie rule). */
void orc_nn_bruteforce(const float* xyz, int64_t m, const float* q,
                       int64_t nq, int32_t* idx, float* d2);

/* ---- align/SolveKabsch (align_icp.cpp:18-71) ----------------------------- */
/* pairs[2c] = src index, pairs[2c+1] = dst index; weights may be NULL.
 * Returns 0 (pose untouched) when n < 3 or m < 3. */
int orc_solve_kabsch(const float* src, int64_t n, const float* dst, int64_t m,
                     const int32_t* pairs, const float* weights, int64_t k,
                     float pose_out[16]);

/* ---- common/centroid (point_cloud_utils.cpp:92-98) ---------------------- */
void orc_centroid(const float* xyz, int64_t n, float out[3]);

/* p = xfm * s with Eigen's operation order (align_icp.cpp:107). */
void orc_transform_points(const float pose[16], const float* xyz, int64_t n,
                          float* out);

/* ---- align/Kabsch pieces (align_icp.cpp:139-151) ------------------------ */
/* Eigen JacobiSVD<Matrix3d>(a, FullU|FullV) restated: a = U diag(s) V^T,
 * s descending.  Matrices column-major. */
void orc_jacobi_svd3(const double a[9], double u[9], double s[3],
                     double v[9]);

/* cov (double, col-major) + means -> pose (R = float(U V^T), reflection fix
 * R.col(2) *= -1, t = dmean - R smean, quaternion round-trip). */
void orc_kabsch_pose(const double cov[9], const float smean[3],
                     const float dmean[3], float pose_out[16]);

/* ---- align/ICP (align_icp.cpp:73-167) ----------------------------------- */
typedef struct {
  /* each array sized max_iter (any may be NULL) */
  float* pose;      /* [max_iter][16] pose after iteration it's update */
  float* cost;      /* [max_iter] fp32 sequential sum of d2 (pre-update)  */
  float* mu;        /* [max_iter] annealing parameter used               */
  double* cov;      /* [max_iter][9] fp64 cross-covariance                */
  float* dmean;     /* [max_iter][3] fp32 mean of matched target points  */
  int32_t* nn_idx0; /* [n] correspondences of iteration 0                 */
  float* nn_d20;    /* [n] squared distances of iteration 0               */
} orc_icp_trace;

/* AlignIcp3d restatement.  tree may be NULL (4-arg overload: builds
 * KDTree3f{dst,16}).  Returns 1 (true) / 0 (false) like the reference; on the
 * early n<3 / m<3 return pose_inout is untouched.  mean_cost may be NULL. */
int orc_align_icp(const float* src, int64_t n, const float* dst, int64_t m,
                  const orc_kdtree* tree, int max_iter, float pose_inout[16],
                  float* mean_cost, orc_icp_trace* trace);

/* Same algorithm with the sums taken in fp64 (sum_mode = 1): centroid and
 * matched-target mean as float(fp64 sum / n), covariance as
 * sum w q u^T - dbar (sum w u)^T in fp64, cost in fp64.  This is the
 * arithmetic the GPU reduction performs; comparing it with sum_mode = 0
 * (the reference's fp32 sequential sums) measures how much the reference's
 * own result moves under a change of summation order. */
int orc_align_icp_ex(const float* src, int64_t n, const float* dst, int64_t m,
                     const orc_kdtree* tree, int max_iter, float pose_inout[16],
                     float* mean_cost, orc_icp_trace* trace, int sum_mode);

/* Threads of orc_align_icp*'s per-point NN loop (OpenMP; default 1).  The
 * sums stay sequential: results are identical for any count. */
void orc_set_threads(int k);

/* One P2POINT_REF iteration's 16 fp64 partial sums over a source range, given
 * the current pose (the quantities the GPU kernels reduce; used by the
 * sharded-host-logic tests):
 *   out[0..8]  = sum w q (s - smean)^T   (row-major r*3+c)
 *   out[9..11] = sum w (s - smean)
 *   out[12..14]= sum q
 *   out[15]    = sum d2                                                       */
void orc_p2point_partials(const float* src, int64_t n, const orc_kdtree* tree,
                          const float* dst, const float pose[16],
                          const float smean[3], float mu, double out[16]);

/* ---- common/normals (point_cloud_utils.cpp:176-216) --------------------- */
/* kNN-PCA normals (self included), then OrientNormals toward viewpoint. */
void orc_compute_normals(const float* xyz, int64_t m, const orc_kdtree* tree,
                         int k, const float viewpoint[3], float* normals);

/* ---- driver/unprojection (librealsense rs2::pointcloud, pinhole) -------- */
/* depth u16 (w*h) -> xyz; invalid (0) pixels -> (0,0,0) (data_source_rs.cpp
 * NaN->0 mapping) when keep_invalid, else dropped.  Returns point count. */
int64_t orc_unproject(const uint16_t* depth, int w, int h, const float K[4],
                      float depth_scale, int keep_invalid, float* xyz);
/* image-grid normals of pyramid level s (restates k_grid_normals) */
int64_t orc_grid_normals(const uint16_t* depth, int w, int h, int s, const float K[4],
                         float depth_scale, int r, const float viewpoint[3], float* normals);
int64_t orc_unproject_strided(const uint16_t* depth, int w, int h, int s, const float K[4],
                              float depth_scale, int keep_invalid, float* xyz);

/* ---- common/RemoveNans (point_cloud_utils.cpp:163-174) ----------------- */
/* Finite points in input order; returns the count (out holds >= n). */
int64_t orc_remove_nans(const float* xyz, int64_t n, float* out);

/* ---- common/DownsampleVoxel (point_cloud_utils.cpp:34-68) --------------- */
/* The first point of every voxel (int)floor(p / voxel_size) (NaN or
 * out-of-int-range -> INT_MIN, x86-64's cast), in ascending input index;
 * returns the count.  The reference emits the same points in unordered_map
 * order. */
int64_t orc_downsample_voxel(const float* xyz, int64_t n, float voxel_size,
                             float* out);

/* ---- f2: GICP (point_cloud_utils.cpp:100-161, align_gicp.cpp:41-163) ---- */
/* ComputeCovariances: covs n x 9 (3x3 col-major each). */
void orc_compute_covariances(const float* xyz, int64_t n, const orc_kdtree* tree,
                             int use_gicp, float* covs);
/* F, and when H/g are non-NULL the robust Gauss-Newton quantities, at the
 * pose (R row-major 3x3, t). */
double orc_gicp_eval(const float* src, int64_t n, const float* dst, const float* src_covs,
                     const float* dst_covs, const int32_t* dst_idx, const double R[9],
                     const double t[3], double H[36], double g[6]);
/* the inner ComputeAlignment (given covariances / correspondences) */
double orc_gicp_solve(const float* src, int64_t n, const float* dst, const float* src_covs,
                      const float* dst_covs, const int32_t* dst_idx, const float seed[16],
                      int max_iter, float pose_out[16], int* iters_out);
/* the 3-argument ComputeAlignment(src, dst, &T) */
double orc_gicp_align(const float* src, int64_t n, const float* dst, int64_t m,
                      int outer_iters, int max_inner, float pose_out[16]);

/* ---- f3: FPFH (fpfh.cpp:20-165,248-300; rst_oracle_fpfh.c) ------------- */
/* ComputeFpfh: out n x 33, input order (normal_k as orc_compute_normals) */
void orc_compute_fpfh(const float* xyz, int64_t n, const float viewpoint[3], int normal_k,
                      float radius, float* out);
/* ComputeMatches: idx n x k (k = 1 or 2), d2 optional */
void orc_compute_matches(const float* src, int64_t n, const float* dst, int64_t m, int k,
                         int32_t* idx, float* d2);

/* ---- f4: CloudAccumulator (rs_replay_app.cpp:76-129) ------------------- */
typedef struct orc_accum orc_accum;
orc_accum* orc_accum_create(float voxel_size);
void orc_accum_free(orc_accum* a);
void orc_accum_add(orc_accum* a, const float pose[16], const float* xyz, int64_t n);
int64_t orc_accum_extract(const orc_accum* a, float* out);

/* ---- build's own point-to-plane mode (no reference counterpart) --------- */
/* Gauss-Newton point-to-plane with the same annealed weight schedule;
 * see DESIGN.md "P2PLANE".  Returns iterations run. */
int orc_align_p2plane(const float* src, int64_t n, const float* dst,
                      const float* dst_normals, int64_t m,
                      const orc_kdtree* tree, int max_iter, float eps,
                      float mu0, float max_dist, float pose_inout[16],
                      float* mean_cost);
/* Its two halves, for the sharded loop (one all-reduce of `out` a step):
 * the normal equations of source points [0, n) at the pose (Rd col-major,
 * td) -- out[0..20] sum w J J^T lower triangle, [21..26] sum w J r, [27]
 * count, [28] sum d2 --, and the solve + pose update on their totals
 * (returns 0 when the system is unusable: the align fails). */
void orc_p2plane_partials(const float* src, int64_t n, const orc_kdtree* tree,
                          const float* dst, const float* dst_normals, const double Rd[9],
                          const double td[3], float mu0, float max_dist, double out[29]);
int orc_p2plane_update(const double tot[29], double Rd[9], double td[3], double* xi_norm,
                       double* cost);

#ifdef __cplusplus
}
#endif
#endif /* RST_ORACLE_H_ */
