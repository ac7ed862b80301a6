/*
 * rst_oracle.c -- CPU ORACLE (test infrastructure only; see rst_oracle.h).
 *
 * Plain-C restatement of the reference's rs_tracker/align ICP path.  Every
 * function cites the reference file:line it follows (paths relative to the
 * reference repository root, rs_tracker/...).  Compiled with
 * -ffp-contract=off so that every float operation rounds exactly as written
 * (the reference builds for baseline x86-64: SSE2, no FMA).
 */
#include "rst_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Distance arithmetic.  nanoflann L2_Adaptor::evalMetric for DIM=3 runs the
 * remainder loop only: result = 0; result += d0*d0; += d1*d1; += d2*d2 with
 * d = query - point (kdtree.hpp:51-57 -> nanoflann).  0 + x == x, so
 * d2 = (dx*dx + dy*dy) + dz*dz. */
static inline float orc_d2(const float* q, const float* p) {
  const float dx = q[0] - p[0];
  const float dy = q[1] - p[1];
  const float dz = q[2] - p[2];
  float r = dx * dx;
  r = r + dy * dy;
  r = r + dz * dz;
  return r;
}

/* lexicographic (d2, idx) "better than" -- the tie rule of this build. */
static inline int orc_better(float d2, int32_t idx, float bd2, int32_t bidx) {
  return (d2 < bd2) || (d2 == bd2 && idx < bidx);
}

/* ------------------------------------------------------------------------ */
/* kd-tree: nanoflann KDTreeSingleIndexAdaptor (kdtree.hpp:27-35) build with
 * middleSplit_ / planeSplit, leaf_max_size as given. */
typedef struct {
  float lo[3], hi[3];
} obox;

typedef struct {
  int32_t child1, child2; /* -1 = leaf */
  int32_t left, right;    /* leaf: [left,right) into vind */
  int32_t divfeat;
  float divlow, divhigh;
} onode;

struct orc_kdtree {
  const float* xyz;
  int64_t m;
  int leaf;
  int32_t* vind;
  onode* nodes;
  int32_t nnodes, cap;
  int32_t root;
  obox root_bbox;
};

static inline float pt(const orc_kdtree* t, int32_t i, int d) {
  return t->xyz[3 * (int64_t)i + d];
}

static int32_t new_node(orc_kdtree* t) {
  if (t->nnodes == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 1024;
    t->nodes = (onode*)realloc(t->nodes, sizeof(onode) * (size_t)t->cap);
  }
  return t->nnodes++;
}

static void compute_minmax(const orc_kdtree* t, const int32_t* ind,
                           int32_t count, int d, float* mn, float* mx) {
  *mn = pt(t, ind[0], d);
  *mx = pt(t, ind[0], d);
  for (int32_t i = 1; i < count; ++i) {
    const float v = pt(t, ind[i], d);
    if (v < *mn) *mn = v;
    if (v > *mx) *mx = v;
  }
}

/* nanoflann planeSplit: two-pass partition around cutval. */
static void plane_split(const orc_kdtree* t, int32_t* ind, int32_t count,
                        int cutfeat, float cutval, int32_t* lim1,
                        int32_t* lim2) {
  int32_t left = 0, right = count - 1;
  for (;;) {
    while (left <= right && pt(t, ind[left], cutfeat) < cutval) ++left;
    while (right && left <= right && pt(t, ind[right], cutfeat) >= cutval)
      --right;
    if (left > right || !right) break;
    int32_t tmp = ind[left];
    ind[left] = ind[right];
    ind[right] = tmp;
    ++left;
    --right;
  }
  *lim1 = left;
  right = count - 1;
  for (;;) {
    while (left <= right && pt(t, ind[left], cutfeat) <= cutval) ++left;
    while (right && left <= right && pt(t, ind[right], cutfeat) > cutval)
      --right;
    if (left > right || !right) break;
    int32_t tmp = ind[left];
    ind[left] = ind[right];
    ind[right] = tmp;
    ++left;
    --right;
  }
  *lim2 = left;
}

/* nanoflann middleSplit_ */
static void middle_split(const orc_kdtree* t, int32_t* ind, int32_t count,
                         int32_t* index, int* cutfeat, float* cutval,
                         const obox* bbox) {
  const float EPS = 0.00001f;
  float max_span = bbox->hi[0] - bbox->lo[0];
  for (int i = 1; i < 3; ++i) {
    const float span = bbox->hi[i] - bbox->lo[i];
    if (span > max_span) max_span = span;
  }
  float max_spread = -1;
  *cutfeat = 0;
  for (int i = 0; i < 3; ++i) {
    const float span = bbox->hi[i] - bbox->lo[i];
    if (span > (1 - EPS) * max_span) {
      float mn, mx;
      compute_minmax(t, ind, count, i, &mn, &mx);
      const float spread = mx - mn;
      if (spread > max_spread) {
        *cutfeat = i;
        max_spread = spread;
      }
    }
  }
  const float split_val = (bbox->lo[*cutfeat] + bbox->hi[*cutfeat]) / 2;
  float mn, mx;
  compute_minmax(t, ind, count, *cutfeat, &mn, &mx);
  if (split_val < mn)
    *cutval = mn;
  else if (split_val > mx)
    *cutval = mx;
  else
    *cutval = split_val;
  int32_t lim1, lim2;
  plane_split(t, ind, count, *cutfeat, *cutval, &lim1, &lim2);
  if (lim1 > count / 2)
    *index = lim1;
  else if (lim2 < count / 2)
    *index = lim2;
  else
    *index = count / 2;
}

/* nanoflann divideTree */
static int32_t divide_tree(orc_kdtree* t, int32_t left, int32_t right,
                           obox* bbox) {
  const int32_t node = new_node(t);
  if ((right - left) <= t->leaf) {
    t->nodes[node].child1 = t->nodes[node].child2 = -1;
    t->nodes[node].left = left;
    t->nodes[node].right = right;
    for (int d = 0; d < 3; ++d) {
      bbox->lo[d] = pt(t, t->vind[left], d);
      bbox->hi[d] = pt(t, t->vind[left], d);
    }
    for (int32_t k = left + 1; k < right; ++k) {
      for (int d = 0; d < 3; ++d) {
        const float v = pt(t, t->vind[k], d);
        if (bbox->lo[d] > v) bbox->lo[d] = v;
        if (bbox->hi[d] < v) bbox->hi[d] = v;
      }
    }
  } else {
    int32_t idx;
    int cutfeat;
    float cutval;
    middle_split(t, t->vind + left, right - left, &idx, &cutfeat, &cutval,
                 bbox);
    t->nodes[node].divfeat = cutfeat;
    obox lb = *bbox;
    lb.hi[cutfeat] = cutval;
    const int32_t c1 = divide_tree(t, left, left + idx, &lb);
    obox rb = *bbox;
    rb.lo[cutfeat] = cutval;
    const int32_t c2 = divide_tree(t, left + idx, right, &rb);
    t->nodes[node].child1 = c1;
    t->nodes[node].child2 = c2;
    t->nodes[node].divlow = lb.hi[cutfeat];
    t->nodes[node].divhigh = rb.lo[cutfeat];
    for (int d = 0; d < 3; ++d) {
      bbox->lo[d] = lb.lo[d] < rb.lo[d] ? lb.lo[d] : rb.lo[d];
      bbox->hi[d] = lb.hi[d] > rb.hi[d] ? lb.hi[d] : rb.hi[d];
    }
  }
  return node;
}

orc_kdtree* orc_kdtree_build(const float* xyz, int64_t m, int leaf_max_size) {
  orc_kdtree* t = (orc_kdtree*)calloc(1, sizeof(orc_kdtree));
  t->xyz = xyz;
  t->m = m;
  t->leaf = leaf_max_size < 1 ? 1 : leaf_max_size;
  t->root = -1;
  if (m <= 0) return t;
  t->vind = (int32_t*)malloc(sizeof(int32_t) * (size_t)m);
  for (int64_t i = 0; i < m; ++i) t->vind[i] = (int32_t)i;
  /* computeBoundingBox */
  for (int d = 0; d < 3; ++d) {
    t->root_bbox.lo[d] = pt(t, 0, d);
    t->root_bbox.hi[d] = pt(t, 0, d);
  }
  for (int64_t k = 1; k < m; ++k)
    for (int d = 0; d < 3; ++d) {
      const float v = pt(t, (int32_t)k, d);
      if (v < t->root_bbox.lo[d]) t->root_bbox.lo[d] = v;
      if (v > t->root_bbox.hi[d]) t->root_bbox.hi[d] = v;
    }
  obox bb = t->root_bbox;
  t->root = divide_tree(t, 0, (int32_t)m, &bb);
  t->root_bbox = bb;
  return t;
}

void orc_kdtree_free(orc_kdtree* t) {
  if (!t) return;
  free(t->vind);
  free(t->nodes);
  free(t);
}

/* k-NN result set: sorted ascending by (d2, idx); k <= 64. */
typedef struct {
  int k, count;
  float d2[64];
  int32_t idx[64];
} orc_rs;

static inline float rs_worst(const orc_rs* rs) {
  return rs->count < rs->k ? FLT_MAX : rs->d2[rs->k - 1];
}

static inline void rs_add(orc_rs* rs, float d2, int32_t idx) {
  /* reference: a point enters only with dist < worst_dist (FLT_MAX when not
   * full), KNNResultSet::addPoint keeps the list sorted */
  if (rs->count == rs->k) {
    if (!orc_better(d2, idx, rs->d2[rs->k - 1], rs->idx[rs->k - 1])) return;
  } else if (!(d2 < FLT_MAX)) {
    return;
  }
  int i = rs->count < rs->k ? rs->count : rs->k - 1;
  while (i > 0 && orc_better(d2, idx, rs->d2[i - 1], rs->idx[i - 1])) {
    rs->d2[i] = rs->d2[i - 1];
    rs->idx[i] = rs->idx[i - 1];
    --i;
  }
  rs->d2[i] = d2;
  rs->idx[i] = idx;
  if (rs->count < rs->k) rs->count++;
}

/* nanoflann searchLevel restated; the box lower bound is recomputed as
 * (dists[0]+dists[1])+dists[2] (monotone => never above any contained
 * point's d2) and a child is entered when bound <= worst, so exact ties are
 * explored and resolved by index. */
static void search_level(const orc_kdtree* t, orc_rs* rs, const float* q,
                         int32_t node, float dists[3]) {
  const onode* nd = &t->nodes[node];
  if (nd->child1 < 0) {
    for (int32_t i = nd->left; i < nd->right; ++i) {
      const int32_t index = t->vind[i];
      const float d2 = orc_d2(q, t->xyz + 3 * (int64_t)index);
      rs_add(rs, d2, index);
    }
    return;
  }
  const int idx = nd->divfeat;
  const float val = q[idx];
  const float diff1 = val - nd->divlow;
  const float diff2 = val - nd->divhigh;
  int32_t best, other;
  float cut_dist;
  if ((diff1 + diff2) < 0) {
    best = nd->child1;
    other = nd->child2;
    cut_dist = (val - nd->divhigh) * (val - nd->divhigh);
  } else {
    best = nd->child2;
    other = nd->child1;
    cut_dist = (val - nd->divlow) * (val - nd->divlow);
  }
  search_level(t, rs, q, best, dists);
  const float dst = dists[idx];
  dists[idx] = cut_dist;
  const float mind = (dists[0] + dists[1]) + dists[2];
  if (mind <= rs_worst(rs)) search_level(t, rs, q, other, dists);
  dists[idx] = dst;
}

static void knn_one(const orc_kdtree* t, const float q[3], int k, orc_rs* rs) {
  rs->k = k;
  rs->count = 0;
  if (t->m <= 0 || t->root < 0) return;
  /* a non-finite query never satisfies dist < worst in the reference */
  if (!(isfinite(q[0]) && isfinite(q[1]) && isfinite(q[2]))) return;
  float dists[3] = {0, 0, 0};
  for (int d = 0; d < 3; ++d) {
    if (q[d] < t->root_bbox.lo[d])
      dists[d] = (q[d] - t->root_bbox.lo[d]) * (q[d] - t->root_bbox.lo[d]);
    if (q[d] > t->root_bbox.hi[d])
      dists[d] = (q[d] - t->root_bbox.hi[d]) * (q[d] - t->root_bbox.hi[d]);
  }
  search_level(t, rs, q, t->root, dists);
}

void orc_kdtree_knn(const orc_kdtree* t, const float q[3], int k,
                    int32_t* idx, float* d2) {
  if (k > 64) k = 64;
  orc_rs rs;
  knn_one(t, q, k, &rs);
  for (int i = 0; i < k; ++i) {
    idx[i] = i < rs.count ? rs.idx[i] : 0;
    d2[i] = i < rs.count ? rs.d2[i] : FLT_MAX;
  }
}

void orc_nn_batch(const orc_kdtree* t, const float* q, int64_t nq,
                  int32_t* idx, float* d2) {
  for (int64_t i = 0; i < nq; ++i) orc_kdtree_knn(t, q + 3 * i, 1, idx + i, d2 + i);
}

void orc_nn_bruteforce(const float* xyz, int64_t m, const float* q,
                       int64_t nq, int32_t* idx, float* d2) {
  for (int64_t i = 0; i < nq; ++i) {
    float bd = FLT_MAX;
    int32_t bi = 0;
    const float* qi = q + 3 * i;
    if (isfinite(qi[0]) && isfinite(qi[1]) && isfinite(qi[2])) {
      for (int64_t j = 0; j < m; ++j) {
        const float d = orc_d2(qi, xyz + 3 * j);
        if (orc_better(d, (int32_t)j, bd, bi) && d < FLT_MAX) {
          bd = d;
          bi = (int32_t)j;
        }
      }
    }
    idx[i] = bi;
    d2[i] = bd;
  }
}

/* ------------------------------------------------------------------------ */
/* ComputeCentroid (point_cloud_utils.cpp:92-98): fp32 sequential sum, then
 * `*centroid *= (1.0 / n)` -- the double is converted to the float Scalar. */
void orc_centroid(const float* xyz, int64_t n, float out[3]) {
  float s0 = 0, s1 = 0, s2 = 0;
  for (int64_t i = 0; i < n; ++i) {
    s0 += xyz[3 * i + 0];
    s1 += xyz[3 * i + 1];
    s2 += xyz[3 * i + 2];
  }
  const float f = (float)(1.0 / (double)n);
  out[0] = s0 * f;
  out[1] = s1 * f;
  out[2] = s2 * f;
}

/* Eigen lazy 3x3 * 3-vector coefficient: redux_novec_unroller splits length
 * 3 as x0 + (x1 + x2). */
static inline float mv_row(const float* R, int r, const float* v) {
  /* R column-major 3x3 */
  const float a0 = R[0 * 3 + r] * v[0];
  const float a1 = R[1 * 3 + r] * v[1];
  const float a2 = R[2 * 3 + r] * v[2];
  return a0 + (a1 + a2);
}

static void pose_split(const float pose[16], float R[9], float t[3]) {
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) R[c * 3 + r] = pose[c * 4 + r];
  for (int r = 0; r < 3; ++r) t[r] = pose[12 + r];
}

static void pose_join(const float R[9], const float t[3], float pose[16]) {
  for (int c = 0; c < 3; ++c) {
    for (int r = 0; r < 3; ++r) pose[c * 4 + r] = R[c * 3 + r];
    pose[c * 4 + 3] = 0.0f;
  }
  for (int r = 0; r < 3; ++r) pose[12 + r] = t[r];
  pose[15] = 1.0f;
}

/* Transform<float,3,Isometry> * Vector3f: res = t; res += linear * v
 * (Eigen transform_right_product_impl), align_icp.cpp:107. */
static inline void xform(const float R[9], const float t[3], const float* s,
                         float* p) {
  for (int r = 0; r < 3; ++r) p[r] = t[r] + mv_row(R, r, s);
}

void orc_transform_points(const float pose[16], const float* xyz, int64_t n,
                          float* out) {
  float R[9], t[3];
  pose_split(pose, R, t);
  for (int64_t i = 0; i < n; ++i) xform(R, t, xyz + 3 * i, out + 3 * i);
}

/* ------------------------------------------------------------------------ */
/* Eigen JacobiSVD<Matrix3d> (square: no QR preconditioner), restated:
 * two-sided Jacobi sweeps with real_2x2_jacobi_svd, then sign fix and
 * descending sort.  Column-major storage a[c*3+r]. */
#define A3(m, r, c) (m)[(c) * 3 + (r)]

typedef struct {
  double c, s;
} jrot;

static jrot jrot_mul(jrot a, jrot b) { /* a * b (real) */
  jrot r;
  r.c = a.c * b.c - a.s * b.s;
  r.s = a.c * b.s + a.s * b.c;
  return r;
}
static jrot jrot_T(jrot a) {
  jrot r = {a.c, -a.s};
  return r;
}

/* apply_rotation_in_the_plane(x, y, j): x' = c x + s y; y' = -s x + c y */
static void rot_rows(double* m, int n, int p, int q, jrot j) {
  for (int i = 0; i < n; ++i) {
    const double xi = A3(m, p, i), yi = A3(m, q, i);
    A3(m, p, i) = j.c * xi + j.s * yi;
    A3(m, q, i) = -j.s * xi + j.c * yi;
  }
}
/* applyOnTheRight(p,q,j) == apply_rotation_in_the_plane(col p, col q, j^T) */
static void rot_cols(double* m, int n, int p, int q, jrot j) {
  const jrot jt = jrot_T(j);
  for (int i = 0; i < n; ++i) {
    const double xi = A3(m, i, p), yi = A3(m, i, q);
    A3(m, i, p) = jt.c * xi + jt.s * yi;
    A3(m, i, q) = -jt.s * xi + jt.c * yi;
  }
}

/* JacobiRotation::makeJacobi(x, y, z) for real scalars */
static jrot make_jacobi(double x, double y, double z) {
  jrot j;
  const double deno = 2.0 * fabs(y);
  if (deno < DBL_MIN) {
    j.c = 1.0;
    j.s = 0.0;
    return j;
  }
  const double tau = (x - z) / deno;
  const double w = sqrt(tau * tau + 1.0);
  double t;
  if (tau > 0)
    t = 1.0 / (tau + w);
  else
    t = 1.0 / (tau - w);
  const double sign_t = t > 0 ? 1.0 : -1.0;
  const double n = 1.0 / sqrt(t * t + 1.0);
  j.s = -sign_t * (y / fabs(y)) * fabs(t) * n;
  j.c = n;
  return j;
}

/* internal::real_2x2_jacobi_svd */
static void real_2x2_jacobi_svd(const double* mat, int p, int q, jrot* jl,
                                jrot* jr) {
  double m00 = A3(mat, p, p), m01 = A3(mat, p, q), m10 = A3(mat, q, p),
         m11 = A3(mat, q, q);
  jrot rot1;
  const double t = m00 + m11;
  const double d = m10 - m01;
  if (fabs(d) < DBL_MIN) {
    rot1.s = 0.0;
    rot1.c = 1.0;
  } else {
    const double u = t / d;
    const double tmp = sqrt(1.0 + u * u);
    rot1.s = 1.0 / tmp;
    rot1.c = u / tmp;
  }
  /* m.applyOnTheLeft(0,1,rot1) on the 2x2 */
  {
    const double x0 = m00, y0 = m10, x1 = m01, y1 = m11;
    m00 = rot1.c * x0 + rot1.s * y0;
    m10 = -rot1.s * x0 + rot1.c * y0;
    m01 = rot1.c * x1 + rot1.s * y1;
    m11 = -rot1.s * x1 + rot1.c * y1;
  }
  (void)m10;
  *jr = make_jacobi(m00, m01, m11);
  *jl = jrot_mul(rot1, jrot_T(*jr));
}

void orc_jacobi_svd3(const double a[9], double u[9], double s[3],
                     double v[9]) {
  const double precision = 2.0 * DBL_EPSILON;
  const double considerAsZero = DBL_MIN;
  double scale = 0;
  for (int i = 0; i < 9; ++i)
    if (fabs(a[i]) > scale || i == 0) scale = fabs(a[i]);
  for (int i = 0; i < 9; ++i) {
    u[i] = (i % 4 == 0) ? 1.0 : 0.0;
    v[i] = (i % 4 == 0) ? 1.0 : 0.0;
  }
  if (!isfinite(scale)) {
    s[0] = s[1] = s[2] = NAN;
    return;
  }
  if (scale == 0) scale = 1.0;
  double w[9];
  for (int i = 0; i < 9; ++i) w[i] = a[i] / scale;
  double maxDiag = 0;
  for (int i = 0; i < 3; ++i)
    if (fabs(A3(w, i, i)) > maxDiag || i == 0) maxDiag = fabs(A3(w, i, i));
  int finished = 0, sweeps = 0;
  while (!finished && sweeps < 100) {
    finished = 1;
    ++sweeps;
    for (int p = 1; p < 3; ++p) {
      for (int q = 0; q < p; ++q) {
        double threshold = precision * maxDiag;
        if (threshold < considerAsZero) threshold = considerAsZero;
        if (fabs(A3(w, p, q)) > threshold || fabs(A3(w, q, p)) > threshold) {
          finished = 0;
          jrot jl, jr;
          real_2x2_jacobi_svd(w, p, q, &jl, &jr);
          rot_rows(w, 3, p, q, jl);
          rot_cols(u, 3, p, q, jrot_T(jl));
          rot_cols(w, 3, p, q, jr);
          rot_cols(v, 3, p, q, jr);
          double mpq = fabs(A3(w, p, p));
          if (fabs(A3(w, q, q)) > mpq) mpq = fabs(A3(w, q, q));
          if (mpq > maxDiag) maxDiag = mpq;
        }
      }
    }
  }
  for (int i = 0; i < 3; ++i) {
    const double ai = A3(w, i, i);
    s[i] = fabs(ai);
    if (ai < 0)
      for (int r = 0; r < 3; ++r) A3(u, r, i) = -A3(u, r, i);
  }
  for (int i = 0; i < 3; ++i) s[i] *= scale;
  for (int i = 0; i < 3; ++i) {
    int pos = i;
    double mx = s[i];
    for (int k = i + 1; k < 3; ++k)
      if (s[k] > mx) {
        mx = s[k];
        pos = k;
      }
    if (mx == 0) break;
    if (pos != i) {
      double tmp = s[i];
      s[i] = s[pos];
      s[pos] = tmp;
      for (int r = 0; r < 3; ++r) {
        tmp = A3(u, r, i);
        A3(u, r, i) = A3(u, r, pos);
        A3(u, r, pos) = tmp;
        tmp = A3(v, r, i);
        A3(v, r, i) = A3(v, r, pos);
        A3(v, r, pos) = tmp;
      }
    }
  }
}

/* Quaternionf(const Matrix3f&) (Eigen quaternionbase_assign_impl<3x3>) then
 * toRotationMatrix(); Translation3f(t) * Quaternionf(R) keeps t unchanged
 * (align_icp.cpp:151). */
static void quat_roundtrip(const float R[9], float Rq[9]) {
  float q[4]; /* x y z w */
  float tr = (A3(R, 0, 0) + A3(R, 1, 1)) + A3(R, 2, 2);
  if (tr > 0.0f) {
    float t = sqrtf(tr + 1.0f);
    q[3] = 0.5f * t;
    t = 0.5f / t;
    q[0] = (A3(R, 2, 1) - A3(R, 1, 2)) * t;
    q[1] = (A3(R, 0, 2) - A3(R, 2, 0)) * t;
    q[2] = (A3(R, 1, 0) - A3(R, 0, 1)) * t;
  } else {
    int i = 0;
    if (A3(R, 1, 1) > A3(R, 0, 0)) i = 1;
    if (A3(R, 2, 2) > A3(R, i, i)) i = 2;
    const int j = (i + 1) % 3;
    const int k = (j + 1) % 3;
    float t = sqrtf(A3(R, i, i) - A3(R, j, j) - A3(R, k, k) + 1.0f);
    q[i] = 0.5f * t;
    t = 0.5f / t;
    q[3] = (A3(R, k, j) - A3(R, j, k)) * t;
    q[j] = (A3(R, j, i) + A3(R, i, j)) * t;
    q[k] = (A3(R, k, i) + A3(R, i, k)) * t;
  }
  const float x = q[0], y = q[1], z = q[2], w = q[3];
  const float tx = 2.0f * x, ty = 2.0f * y, tz = 2.0f * z;
  const float twx = tx * w, twy = ty * w, twz = tz * w;
  const float txx = tx * x, txy = ty * x, txz = tz * x;
  const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
  A3(Rq, 0, 0) = 1.0f - (tyy + tzz);
  A3(Rq, 0, 1) = txy - twz;
  A3(Rq, 0, 2) = txz + twy;
  A3(Rq, 1, 0) = txy + twz;
  A3(Rq, 1, 1) = 1.0f - (txx + tzz);
  A3(Rq, 1, 2) = tyz - twx;
  A3(Rq, 2, 0) = txz - twy;
  A3(Rq, 2, 1) = tyz + twx;
  A3(Rq, 2, 2) = 1.0f - (txx + tyy);
}

/* Matrix3f::determinant (bruteforce_det3_helper) */
static float det3f(const float* m) {
  const float d0 =
      A3(m, 0, 0) * (A3(m, 1, 1) * A3(m, 2, 2) - A3(m, 1, 2) * A3(m, 2, 1));
  const float d1 =
      A3(m, 0, 1) * (A3(m, 1, 0) * A3(m, 2, 2) - A3(m, 1, 2) * A3(m, 2, 0));
  const float d2 =
      A3(m, 0, 2) * (A3(m, 1, 0) * A3(m, 2, 1) - A3(m, 1, 1) * A3(m, 2, 0));
  return (d0 - d1) + d2;
}

/* align_icp.cpp:139-151 */
void orc_kabsch_pose(const double cov[9], const float smean[3],
                     const float dmean[3], float pose_out[16]) {
  double U[9], S[3], V[9];
  orc_jacobi_svd3(cov, U, S, V);
  float R[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      /* (U * V^T)(r,c) = sum_k U(r,k) V(c,k) */
      const double a0 = A3(U, r, 0) * A3(V, c, 0);
      const double a1 = A3(U, r, 1) * A3(V, c, 1);
      const double a2 = A3(U, r, 2) * A3(V, c, 2);
      A3(R, r, c) = (float)(a0 + (a1 + a2));
    }
  if (det3f(R) < 0) {
    for (int r = 0; r < 3; ++r) A3(R, r, 2) *= -1.0f;
  }
  float t[3];
  for (int r = 0; r < 3; ++r) t[r] = dmean[r] - mv_row(R, r, smean);
  float Rq[9];
  quat_roundtrip(R, Rq);
  pose_join(Rq, t, pose_out);
}

/* ------------------------------------------------------------------------ */
/* SolveKabsch (align_icp.cpp:18-71): fp32 sequential means over the pairs
 * (:27-34), cov += w * double(float((q - dbar)(s - sbar)^T)) (:36-54), then
 * the Kabsch of :58-69 (same as the ICP's :139-151). */
int orc_solve_kabsch(const float* src, int64_t n, const float* dst, int64_t m,
                     const int32_t* pairs, const float* weights, int64_t k,
                     float pose_out[16]) {
  if (n < 3 || m < 3) return 0; /* :22-24 */
  float sm[3] = {0.f, 0.f, 0.f}, dm[3] = {0.f, 0.f, 0.f};
  for (int64_t c = 0; c < k; ++c)
    for (int a = 0; a < 3; ++a) {
      sm[a] += src[3 * (int64_t)pairs[2 * c] + a];
      dm[a] += dst[3 * (int64_t)pairs[2 * c + 1] + a];
    }
  const float fk = (float)k; /* Vector3f /= size_t */
  for (int a = 0; a < 3; ++a) {
    sm[a] /= fk;
    dm[a] /= fk;
  }
  double cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t c = 0; c < k; ++c) {
    const float* s = src + 3 * (int64_t)pairs[2 * c];
    const float* q = dst + 3 * (int64_t)pairs[2 * c + 1];
    const float u[3] = {s[0] - sm[0], s[1] - sm[1], s[2] - sm[2]};
    const float v[3] = {q[0] - dm[0], q[1] - dm[1], q[2] - dm[2]};
    const double w = weights ? (double)weights[c] : 1.0;
    for (int r = 0; r < 3; ++r)
      for (int cc = 0; cc < 3; ++cc) A3(cov, r, cc) += w * (double)(v[r] * u[cc]);
  }
  orc_kabsch_pose(cov, sm, dm, pose_out);
  return 1;
}

/* ------------------------------------------------------------------------ */
/* OpenMP threads of the per-point NN loop (1 = the reference's single
 * thread; the all-cores CPU baseline sets more).  Results do not depend on it. */
static int g_threads = 1;
void orc_set_threads(int k) { g_threads = k < 1 ? 1 : k; }

/* AlignIcp3d (align_icp.cpp:73-161; 4-arg overload :163-167) */
int orc_align_icp(const float* src, int64_t n, const float* dst, int64_t m,
                  const orc_kdtree* tree, int max_iter, float pose_inout[16],
                  float* mean_cost, orc_icp_trace* trace) {
  return orc_align_icp_ex(src, n, dst, m, tree, max_iter, pose_inout, mean_cost,
                          trace, 0);
}

int orc_align_icp_ex(const float* src, int64_t n, const float* dst, int64_t m,
                     const orc_kdtree* tree, int max_iter, float pose_inout[16],
                     float* mean_cost, orc_icp_trace* trace, int sum_mode) {
  if (n < 3 || m < 3) return 0; /* :77-79, transform untouched */
  orc_kdtree* own = NULL;
  if (!tree) {
    own = orc_kdtree_build(dst, m, 16); /* :165 KDTree3f{dst,16} */
    tree = own;
  }
  float R[9], t[3];
  pose_split(pose_inout, R, t); /* :82 xfm = *transform */
  float smean[3];
  if (sum_mode == 0) {
    orc_centroid(src, n, smean); /* :85-86 */
  } else {
    double a[3] = {0, 0, 0};
    for (int64_t i = 0; i < n; ++i)
      for (int d = 0; d < 3; ++d) a[d] += (double)src[3 * i + d];
    for (int d = 0; d < 3; ++d) smean[d] = (float)(a[d] / (double)n);
  }
  int32_t* nbrs = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  float* weights = (float*)malloc(sizeof(float) * (size_t)n);
  float* d2s = (float*)malloc(sizeof(float) * (size_t)n);
  float cost = 0.0f;
  float mu = 1.0f;
  for (int iter = 0; iter < max_iter; ++iter) {
    if (iter > 0 && iter % 8 == 0) mu /= 1.4f; /* :96-98 */
    float dmean[3] = {0.0f, 0.0f, 0.0f};
    double dsum[3] = {0, 0, 0}, csum = 0;
    cost = 0.0f;
    /* :107,112 -- the per-point transform and exact 1-NN are independent of
     * each other: with orc_set_threads(k > 1) they run on k OpenMP threads
     * (the all-cores CPU baseline); every sum below stays sequential in i,
     * so the result is identical for any thread count */
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int64_t i = 0; i < n; ++i) {
      float p[3];
      xform(R, t, src + 3 * i, p);
      int32_t j = 0;
      float d2 = 0;
      orc_kdtree_knn(tree, p, 1, &j, &d2);
      nbrs[i] = j;
      d2s[i] = d2;
    }
    for (int64_t i = 0; i < n; ++i) { /* :105-121 */
      const int32_t j = nbrs[i];
      const float d2 = d2s[i];
      cost += d2;
      csum += (double)d2;
      nbrs[i] = j;
      const float l_pq_rt = mu / (d2 + mu);
      const float l_pq = l_pq_rt * l_pq_rt;
      weights[i] = l_pq;
      for (int d = 0; d < 3; ++d) {
        dmean[d] += dst[3 * (int64_t)j + d];
        dsum[d] += (double)dst[3 * (int64_t)j + d];
      }
      if (iter == 0 && trace) {
        if (trace->nn_idx0) trace->nn_idx0[i] = j;
        if (trace->nn_d20) trace->nn_d20[i] = d2;
      }
    }
    double cov[9] = {0};
    if (sum_mode == 0) {
      const float nf = (float)n; /* :122 dst_mean /= n (int -> Scalar) */
      dmean[0] = dmean[0] / nf;
      dmean[1] = dmean[1] / nf;
      dmean[2] = dmean[2] / nf;
      for (int64_t i = 0; i < n; ++i) { /* :125-136 */
        const float* q = dst + 3 * (int64_t)nbrs[i];
        const float* s = src + 3 * i;
        float a[3], b[3];
        for (int r = 0; r < 3; ++r) a[r] = weights[i] * (q[r] - dmean[r]);
        for (int c = 0; c < 3; ++c) b[c] = s[c] - smean[c];
        for (int c = 0; c < 3; ++c)
          for (int r = 0; r < 3; ++r) A3(cov, r, c) += (double)(b[c] * a[r]);
      }
    } else {
      for (int d = 0; d < 3; ++d) dmean[d] = (float)(dsum[d] / (double)n);
      cost = (float)csum;
      double wqu[9] = {0}, wu[3] = {0};
      for (int64_t i = 0; i < n; ++i) {
        const float* q = dst + 3 * (int64_t)nbrs[i];
        const float* s = src + 3 * i;
        const double w = (double)weights[i];
        double u[3];
        for (int c = 0; c < 3; ++c) u[c] = (double)(s[c] - smean[c]);
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) wqu[r * 3 + c] += w * (double)q[r] * u[c];
        for (int c = 0; c < 3; ++c) wu[c] += w * u[c];
      }
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
          A3(cov, r, c) = wqu[r * 3 + c] - (double)dmean[r] * wu[c];
    }
    float pose[16];
    orc_kabsch_pose(cov, smean, dmean, pose); /* :139-151 */
    pose_split(pose, R, t);
    if (trace) {
      if (trace->pose) memcpy(trace->pose + 16 * iter, pose, sizeof(pose));
      if (trace->cost) trace->cost[iter] = cost;
      if (trace->mu) trace->mu[iter] = mu;
      if (trace->cov) memcpy(trace->cov + 9 * iter, cov, sizeof(cov));
      if (trace->dmean) memcpy(trace->dmean + 3 * iter, dmean, sizeof(dmean));
    }
  }
  pose_join(R, t, pose_inout); /* :156 */
  const float mc = sqrtf(cost / (float)n); /* :157 */
  if (mean_cost) *mean_cost = mc;
  free(nbrs);
  free(weights);
  free(d2s);
  if (own) orc_kdtree_free(own);
  return mc < 10000.0f; /* :160 */
}

void orc_p2point_partials(const float* src, int64_t n, const orc_kdtree* tree,
                          const float* dst, const float pose[16],
                          const float smean[3], float mu, double out[16]) {
  float R[9], t[3];
  pose_split(pose, R, t);
  for (int k = 0; k < 16; ++k) out[k] = 0;
  for (int64_t i = 0; i < n; ++i) {
    float p[3];
    xform(R, t, src + 3 * i, p);
    int32_t j = 0;
    float d2 = 0;
    orc_kdtree_knn(tree, p, 1, &j, &d2);
    const float l = mu / (d2 + mu);
    const double w = (double)(l * l);
    const float* q = dst + 3 * (int64_t)j;
    double u[3];
    for (int c = 0; c < 3; ++c) u[c] = (double)(src[3 * i + c] - smean[c]);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) out[r * 3 + c] += w * (double)q[r] * u[c];
    for (int c = 0; c < 3; ++c) out[9 + c] += w * u[c];
    for (int r = 0; r < 3; ++r) out[12 + r] += (double)q[r];
    out[15] += (double)d2;
  }
}

/* ------------------------------------------------------------------------ */
/* 3x3 symmetric eigen (cyclic Jacobi, double): eigenvector of the smallest
 * eigenvalue.  Stands in for Eigen::SelfAdjointEigenSolver<MatrixXf>
 * eigenvectors().col(0) (point_cloud_utils.cpp:201-202); the sign is
 * arbitrary in both and fixed by OrientNormals. */
static void sym3_min_eigvec(const double a_in[9], double out[3]) {
  double a[9], v[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  memcpy(a, a_in, sizeof(a));
  for (int sweep = 0; sweep < 60; ++sweep) {
    const double off = A3(a, 0, 1) * A3(a, 0, 1) + A3(a, 0, 2) * A3(a, 0, 2) +
                       A3(a, 1, 2) * A3(a, 1, 2);
    if (off < 1e-300) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        const double apq = A3(a, p, q);
        if (fabs(apq) < 1e-300) continue;
        const double theta = (A3(a, q, q) - A3(a, p, p)) / (2.0 * apq);
        const double tt = (theta >= 0 ? 1.0 : -1.0) /
                          (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
        for (int k = 0; k < 3; ++k) { /* A <- J^T A J */
          const double akp = A3(a, k, p), akq = A3(a, k, q);
          A3(a, k, p) = c * akp - s * akq;
          A3(a, k, q) = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          const double apk = A3(a, p, k), aqk = A3(a, q, k);
          A3(a, p, k) = c * apk - s * aqk;
          A3(a, q, k) = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {
          const double vkp = A3(v, k, p), vkq = A3(v, k, q);
          A3(v, k, p) = c * vkp - s * vkq;
          A3(v, k, q) = s * vkp + c * vkq;
        }
      }
  }
  int mi = 0;
  for (int i = 1; i < 3; ++i)
    if (A3(a, i, i) < A3(a, mi, mi)) mi = i;
  double nrm = 0;
  for (int r = 0; r < 3; ++r) nrm += A3(v, r, mi) * A3(v, r, mi);
  nrm = sqrt(nrm);
  for (int r = 0; r < 3; ++r) out[r] = A3(v, r, mi) / nrm;
}

/* ComputeNormals + OrientNormals (point_cloud_utils.cpp:176-216) */
void orc_compute_normals(const float* xyz, int64_t m, const orc_kdtree* tree,
                         int k, const float viewpoint[3], float* normals) {
  int32_t oi[64];
  float od[64];
  if (k > 64) k = 64;
  const float kf = (float)k;
  for (int64_t i = 0; i < m; ++i) {
    const float* p = xyz + 3 * i;
    orc_kdtree_knn(tree, p, k, oi, od);
    float c[3] = {0, 0, 0};
    for (int j = 0; j < k; ++j)
      for (int d = 0; d < 3; ++d) c[d] += xyz[3 * (int64_t)oi[j] + d];
    for (int d = 0; d < 3; ++d) c[d] = c[d] / kf; /* centroid /= num_neighbors */
    float cov[9] = {0};
    for (int j = 0; j < k; ++j) {
      float dl[3];
      for (int d = 0; d < 3; ++d) dl[d] = xyz[3 * (int64_t)oi[j] + d] - c[d];
      for (int cc = 0; cc < 3; ++cc)
        for (int r = 0; r < 3; ++r) A3(cov, r, cc) += dl[r] * dl[cc];
    }
    double cd[9], nv[3];
    for (int q = 0; q < 9; ++q) cd[q] = (double)cov[q];
    sym3_min_eigvec(cd, nv);
    float n[3] = {(float)nv[0], (float)nv[1], (float)nv[2]};
    /* OrientNormals: ray = p - viewpoint; flip if ray.dot(n) > 0 */
    const float ray[3] = {p[0] - viewpoint[0], p[1] - viewpoint[1],
                          p[2] - viewpoint[2]};
    const float dot = ray[0] * n[0] + (ray[1] * n[1] + ray[2] * n[2]);
    if (dot > 0) {
      n[0] = -n[0];
      n[1] = -n[1];
      n[2] = -n[2];
    }
    normals[3 * i + 0] = n[0];
    normals[3 * i + 1] = n[1];
    normals[3 * i + 2] = n[2];
  }
}

/* Image-grid normals (the build's point-to-plane perf mode; no reference
 * counterpart -- restates k_grid_normals, query.hip): per valid pixel of
 * pyramid level s, the valid points of its (2r+1)^2 level-pixel window
 * within 5 r s z / fx of it (window order: rows, then columns), fp32
 * centroid and covariance as ComputeNormals (point_cloud_utils.cpp:186-198),
 * smallest eigenvector, OrientNormals (:206-216); < 3 points: the unit ray
 * towards the viewpoint.  Output in unproject order (valid pixels,
 * row-major). */
int64_t orc_grid_normals(const uint16_t* depth, int w, int h, int s, const float K[4],
                         float depth_scale, int r, const float viewpoint[3], float* normals) {
  const int wl = (w + s - 1) / s, hl = (h + s - 1) / s;
  float* g = (float*)malloc(sizeof(float) * 3 * (size_t)wl * hl);
  if (!g) return -1;
  orc_unproject_strided(depth, w, h, s, K, depth_scale, 1, g);
  int64_t k = 0;
  for (int v = 0; v < hl; ++v)
    for (int u = 0; u < wl; ++u) {
      const float* p = g + 3 * ((int64_t)v * wl + u);
      if (depth[(int64_t)v * s * w + (int64_t)u * s] == 0) continue;
      const float reach = 5.0f * (float)r * (float)s * p[2] / fabsf(K[0]);
      const float reach2 = reach * reach;
      float c[3] = {0, 0, 0}, cov[6] = {0, 0, 0, 0, 0, 0};
      int cnt = 0;
      for (int pass = 0; pass < 2; ++pass) {
        for (int dv = -r; dv <= r; ++dv)
          for (int du = -r; du <= r; ++du) {
            const int uu = u + du, vv = v + dv;
            if (uu < 0 || vv < 0 || uu >= wl || vv >= hl) continue;
            if (depth[(int64_t)vv * s * w + (int64_t)uu * s] == 0) continue;
            const float* q = g + 3 * ((int64_t)vv * wl + uu);
            const float ex = q[0] - p[0], ey = q[1] - p[1], ez = q[2] - p[2];
            if ((ex * ex + ey * ey) + ez * ez > reach2) continue;
            if (pass == 0) {
              c[0] += q[0];
              c[1] += q[1];
              c[2] += q[2];
              ++cnt;
            } else {
              const float dx = q[0] - c[0], dy = q[1] - c[1], dz = q[2] - c[2];
              cov[0] += dx * dx; cov[1] += dx * dy; cov[2] += dx * dz;
              cov[3] += dy * dy; cov[4] += dy * dz; cov[5] += dz * dz;
            }
          }
        if (pass == 0) {
          if (cnt < 3) break;
          const float kf = (float)cnt;
          for (int d = 0; d < 3; ++d) c[d] = c[d] / kf;
        }
      }
      float n[3];
      if (cnt >= 3) {
        const double cd[9] = {cov[0], cov[1], cov[2], cov[1], cov[3], cov[4], cov[2], cov[4], cov[5]};
        double nv[3];
        sym3_min_eigvec(cd, nv);
        n[0] = (float)nv[0];
        n[1] = (float)nv[1];
        n[2] = (float)nv[2];
      } else {
        n[0] = p[0] - viewpoint[0];
        n[1] = p[1] - viewpoint[1];
        n[2] = p[2] - viewpoint[2];
        const float l = sqrtf((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]);
        const float il = l > 0.f ? 1.0f / l : 0.f;
        n[0] *= il;
        n[1] *= il;
        n[2] = l > 0.f ? n[2] * il : 1.f;
      }
      const float ray[3] = {p[0] - viewpoint[0], p[1] - viewpoint[1], p[2] - viewpoint[2]};
      if (ray[0] * n[0] + (ray[1] * n[1] + ray[2] * n[2]) > 0) {
        n[0] = -n[0];
        n[1] = -n[1];
        n[2] = -n[2];
      }
      normals[3 * k + 0] = n[0];
      normals[3 * k + 1] = n[1];
      normals[3 * k + 2] = n[2];
      ++k;
    }
  free(g);
  return k;
}

/* ------------------------------------------------------------------------ */
/* librealsense rs2_deproject_pixel_to_point, no distortion:
 *   x = (u - ppx)/fx; y = (v - ppy)/fy; P = (z*x, z*y, z), z = scale*d. */
int64_t orc_unproject(const uint16_t* depth, int w, int h, const float K[4],
                      float depth_scale, int keep_invalid, float* xyz) {
  return orc_unproject_strided(depth, w, h, 1, K, depth_scale, keep_invalid, xyz);
}

/* Pyramid level of stride s (BASELINE configs[4]; no reference
 * counterpart): pixels (u, v) with u % s == 0 and v % s == 0, row-major,
 * deprojected with the full image's intrinsics. */
int64_t orc_unproject_strided(const uint16_t* depth, int w, int h, int s, const float K[4],
                              float depth_scale, int keep_invalid, float* xyz) {
  const float fx = K[0], fy = K[1], cx = K[2], cy = K[3];
  int64_t k = 0;
  for (int v = 0; v < h; v += s)
    for (int u = 0; u < w; u += s) {
      const uint16_t d = depth[(int64_t)v * w + u];
      if (d == 0 && !keep_invalid) continue;
      const float z = depth_scale * (float)d;
      const float x = ((float)u - cx) / fx;
      const float y = ((float)v - cy) / fy;
      xyz[3 * k + 0] = z * x;
      xyz[3 * k + 1] = z * y;
      xyz[3 * k + 2] = z;
      ++k;
    }
  return k;
}

/* ------------------------------------------------------------------------ */
/* Build's own point-to-plane Gauss-Newton (DESIGN.md "P2PLANE").
 *   r = n.(p - q)  with p = R s + t (reference op order), q, n at the NN;
 *   w = (mu/(r^2+mu))^2, correspondences with d2 > max_dist^2 rejected;
 *   J = [p x n ; n];  A = sum w J J^T,  b = sum w J r;  A xi = -b;
 *   T <- exp([w]x) T + v  (left update), stop when |xi| < eps. */
static void rodrigues(const double w[3], double R[9]) {
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  double K[9] = {0, w[2], -w[1], -w[2], 0, w[0], w[1], -w[0], 0};
  double a, b;
  if (th < 1e-12) {
    a = 1.0;
    b = 0.5;
  } else {
    a = sin(th) / th;
    b = (1.0 - cos(th)) / (th * th);
  }
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) {
      double kk = 0;
      for (int l = 0; l < 3; ++l) kk += A3(K, r, l) * A3(K, l, c);
      A3(R, r, c) = (r == c ? 1.0 : 0.0) + a * A3(K, r, c) + b * kk;
    }
}

static int chol_solve6(const double A[36], const double b[6], double x[6]) {
  double L[36] = {0};
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = A[i * 6 + j];
      for (int k = 0; k < j; ++k) s -= L[i * 6 + k] * L[j * 6 + k];
      if (i == j) {
        if (!(s > 0)) return 0;
        L[i * 6 + i] = sqrt(s);
      } else {
        L[i * 6 + j] = s / L[j * 6 + j];
      }
    }
  double y[6];
  for (int i = 0; i < 6; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[i * 6 + k] * y[k];
    y[i] = s / L[i * 6 + i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < 6; ++k) s -= L[k * 6 + i] * x[k];
    x[i] = s / L[i * 6 + i];
  }
  return 1;
}

/* One iteration's normal equations over source points [0, n) at the pose
 * (Rd, td) (column-major 3x3 + 3, double; rounded to float for the
 * transform): out[0..20] = sum w J J^T (lower triangle, row a, c <= a),
 * out[21..26] = sum w J r, out[27] = count, out[28] = sum d2, summed in
 * ascending i.  A shard's partials: the sharded loop all-reduces them (the
 * north_star's per-iteration RCCL all-reduce of the 6x6 / 6x1 system). */
void orc_p2plane_partials(const float* src, int64_t n, const orc_kdtree* tree,
                          const float* dst, const float* dst_normals, const double Rd[9],
                          const double td[3], float mu0, float max_dist, double out[29]) {
  float R[9], t[3];
  for (int q = 0; q < 9; ++q) R[q] = (float)Rd[q];
  for (int r = 0; r < 3; ++r) t[r] = (float)td[r];
  const float md2 = max_dist > 0 ? max_dist * max_dist : FLT_MAX;
  double A[21] = {0}, b[6] = {0}, cnt = 0, d2sum = 0;
  for (int64_t i = 0; i < n; ++i) {
    float p[3];
    xform(R, t, src + 3 * i, p);
    int32_t j = 0;
    float d2 = 0;
    orc_kdtree_knn(tree, p, 1, &j, &d2);
    if (!(d2 <= md2)) continue;
    const float* q = dst + 3 * (int64_t)j;
    const float* nn = dst_normals + 3 * (int64_t)j;
    const float e0 = p[0] - q[0], e1 = p[1] - q[1], e2 = p[2] - q[2];
    const float r = (nn[0] * e0 + nn[1] * e1) + nn[2] * e2;
    const double dr = (double)r;
    const double l = (double)mu0 / (dr * dr + (double)mu0);
    const double w = l * l;
    const double P[3] = {p[0], p[1], p[2]}, N[3] = {nn[0], nn[1], nn[2]};
    const double J[6] = {P[1] * N[2] - P[2] * N[1], P[2] * N[0] - P[0] * N[2],
                         P[0] * N[1] - P[1] * N[0], N[0], N[1], N[2]};
    for (int a = 0, k = 0; a < 6; ++a) {
      for (int c = 0; c <= a; ++c, ++k) A[k] += w * J[a] * J[c];
      b[a] += w * J[a] * dr;
    }
    cnt += 1.0;
    d2sum += (double)d2;
  }
  memcpy(out, A, sizeof(A));
  memcpy(out + 21, b, sizeof(b));
  out[27] = cnt;
  out[28] = d2sum;
}

/* The solve every rank runs on the (all-reduced) normal equations: A xi = -b
 * by Cholesky, T <- exp([w]x) T + v.  Returns 0 when the system is
 * unusable (< 6 correspondences, not positive definite): the align fails. */
int orc_p2plane_update(const double tot[29], double Rd[9], double td[3], double* xi_norm,
                       double* cost) {
  if (tot[27] < 6) return 0;
  double A[36], nb[6], xi[6];
  for (int a = 0, k = 0; a < 6; ++a)
    for (int c = 0; c <= a; ++c, ++k) A[a * 6 + c] = A[c * 6 + a] = tot[k];
  for (int a = 0; a < 6; ++a) nb[a] = -tot[21 + a];
  if (!chol_solve6(A, nb, xi)) return 0;
  double dR[9];
  rodrigues(xi, dR);
  double nR[9], nt[3];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) {
      double s = 0;
      for (int l2 = 0; l2 < 3; ++l2) s += A3(dR, r, l2) * A3(Rd, l2, c);
      A3(nR, r, c) = s;
    }
  for (int r = 0; r < 3; ++r) {
    double s = 0;
    for (int l2 = 0; l2 < 3; ++l2) s += A3(dR, r, l2) * td[l2];
    nt[r] = s + xi[3 + r];
  }
  memcpy(Rd, nR, sizeof(nR));
  memcpy(td, nt, sizeof(nt));
  *cost = sqrt(tot[28] / tot[27]);
  double nx = 0;
  for (int a = 0; a < 6; ++a) nx += xi[a] * xi[a];
  *xi_norm = sqrt(nx);
  return 1;
}

int orc_align_p2plane(const float* src, int64_t n, const float* dst,
                      const float* dst_normals, int64_t m,
                      const orc_kdtree* tree, int max_iter, float eps,
                      float mu0, float max_dist, float pose_inout[16],
                      float* mean_cost) {
  if (n < 6 || m < 3) return -1;
  orc_kdtree* own = NULL;
  if (!tree) {
    own = orc_kdtree_build(dst, m, 16);
    tree = own;
  }
  double Rd[9], td[3];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) Rd[c * 3 + r] = pose_inout[c * 4 + r];
  for (int r = 0; r < 3; ++r) td[r] = pose_inout[12 + r];
  int it = 0, ok = 1;
  double last_cost = 0;
  for (it = 0; it < max_iter;) {
    double tot[29], xn = 0;
    orc_p2plane_partials(src, n, tree, dst, dst_normals, Rd, td, mu0, max_dist, tot);
    if (!orc_p2plane_update(tot, Rd, td, &xn, &last_cost)) {
      ok = 0;
      break;
    }
    ++it;
    if (xn < (double)eps) break;
  }
  if (ok) {
    for (int c = 0; c < 3; ++c) {
      for (int r = 0; r < 3; ++r) pose_inout[c * 4 + r] = (float)Rd[c * 3 + r];
      pose_inout[c * 4 + 3] = 0.0f;
    }
    for (int r = 0; r < 3; ++r) pose_inout[12 + r] = (float)td[r];
    pose_inout[15] = 1.0f;
    if (mean_cost) *mean_cost = (float)last_cost;
  }
  if (own) orc_kdtree_free(own);
  return ok ? it : -1;
}

/* ---- common/RemoveNans (point_cloud_utils.cpp:163-174) ------------------- */
int64_t orc_remove_nans(const float* xyz, int64_t n, float* out) {
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float* p = xyz + 3 * i;
    if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue; /* :167 allFinite */
    out[3 * m + 0] = p[0];
    out[3 * m + 1] = p[1];
    out[3 * m + 2] = p[2];
    ++m;
  }
  return m;
}

/* ---- common/DownsampleVoxel (point_cloud_utils.cpp:34-68) --------------- */
/* (point / voxel_size).floor().cast<int>() (:41-42) per axis; the cast of a
 * NaN / out-of-range float is what x86-64 cvttss2si returns, INT_MIN. */
static int orc_vox_coord(float x, float v) {
  const float q = floorf(x / v);
  return (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT_MIN;
}

int64_t orc_downsample_voxel(const float* xyz, int64_t n, float voxel_size, float* out) {
  /* the set of voxels seen so far (:43-46: emplace only when new, so each
   * voxel keeps its FIRST point); open addressing over (ix,iy,iz) */
  int64_t cap = 16;
  while (cap < 2 * n) cap <<= 1;
  int32_t* keys = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)cap);
  uint8_t* used = (uint8_t*)calloc((size_t)cap, 1);
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float* p = xyz + 3 * i;
    const int k0 = orc_vox_coord(p[0], voxel_size), k1 = orc_vox_coord(p[1], voxel_size),
              k2 = orc_vox_coord(p[2], voxel_size);
    uint64_t h = ((uint64_t)(uint32_t)k0 * 73856093u) ^ ((uint64_t)(uint32_t)k1 * 19349663u) ^
                 ((uint64_t)(uint32_t)k2 * 83492791u);
    h ^= h >> 17;
    int64_t s = (int64_t)(h & (uint64_t)(cap - 1));
    int found = 0;
    while (used[s]) {
      if (keys[3 * s] == k0 && keys[3 * s + 1] == k1 && keys[3 * s + 2] == k2) {
        found = 1;
        break;
      }
      s = (s + 1) & (cap - 1);
    }
    if (found) continue;
    used[s] = 1;
    keys[3 * s] = k0;
    keys[3 * s + 1] = k1;
    keys[3 * s + 2] = k2;
    /* emitted in first-seen (= ascending index) order; the reference emits
     * the same set in unordered_map iteration order (:54-57, :63-66) */
    out[3 * m + 0] = p[0];
    out[3 * m + 1] = p[1];
    out[3 * m + 2] = p[2];
    ++m;
  }
  free(keys);
  free(used);
  return m;
}

/* ==== f2: GICP (point_cloud_utils.cpp:100-161, align_gicp.cpp:41-163) ===== */

/* ComputeCovariances: 33-NN (self included, first result dropped), fp32
 * centroid of the 32 neighbours in result order, fp32 sum of outer
 * products, / 31 (:117-159); use_gicp: cov <- U diag(1, 1, 1e-2) U^T with U
 * the singular vectors of cov (:139-155), here I - (1 - 1e-2) u3 u3^T in
 * fp64 (u3 = the smallest singular vector; independent of U's signs). */
void orc_compute_covariances(const float* xyz, int64_t n, const orc_kdtree* tree,
                             int use_gicp, float* covs) {
  int32_t idx[33];
  float d2[33];
  for (int64_t i = 0; i < n; ++i) {
    orc_kdtree_knn(tree, xyz + 3 * i, 33, idx, d2);
    float c[3] = {0.f, 0.f, 0.f};
    for (int j = 1; j < 33; ++j)
      for (int r = 0; r < 3; ++r) c[r] += xyz[3 * (int64_t)idx[j] + r];
    for (int r = 0; r < 3; ++r) c[r] /= 32.0f;
    float cov[9] = {0};
    for (int j = 1; j < 33; ++j) {
      float dl[3];
      for (int r = 0; r < 3; ++r) dl[r] = xyz[3 * (int64_t)idx[j] + r] - c[r];
      for (int cc = 0; cc < 3; ++cc)
        for (int r = 0; r < 3; ++r) cov[cc * 3 + r] += dl[r] * dl[cc];
    }
    float* o = covs + 9 * i;
    if (use_gicp) {
      double a[9], u[9], s[3], v[9];
      for (int k = 0; k < 9; ++k) a[k] = cov[k];
      orc_jacobi_svd3(a, u, s, v);
      const double* u3 = u + 6; /* column 2: smallest singular value */
      for (int cc = 0; cc < 3; ++cc)
        for (int r = 0; r < 3; ++r)
          o[cc * 3 + r] = (float)((r == cc ? 1.0 : 0.0) - (1.0 - 1e-2) * u3[r] * u3[cc]);
    } else {
      for (int k = 0; k < 9; ++k) o[k] = cov[k] / 31.0f;
    }
  }
}

/* symmetric 3x3 eigen-decomposition, cyclic Jacobi (fp64); a row-major
 * scalars, V columns = eigenvectors */
static void gicp_sym_eig3(const double A[9], double lam[3], double V[9]) {
  double a[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) a[r][c] = A[3 * r + c];
  double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
  for (int sweep = 0; sweep < 12; ++sweep) {
    const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
    const double dg = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
    if (!(off > 1e-32 * dg)) break;
    for (int k = 0; k < 3; ++k) {
      const int p = P[k], q = Q[k];
      const double apq = a[p][q];
      if (apq == 0.0) continue;
      const double th = (a[q][q] - a[p][p]) / (2.0 * apq);
      const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
      const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
      for (int r = 0; r < 3; ++r) { /* A <- A J (columns p, q) */
        const double arp = a[r][p], arq = a[r][q];
        a[r][p] = c * arp - s * arq;
        a[r][q] = s * arp + c * arq;
      }
      for (int r = 0; r < 3; ++r) { /* A <- J^T A (rows p, q) */
        const double apr = a[p][r], aqr = a[q][r];
        a[p][r] = c * apr - s * aqr;
        a[q][r] = s * apr + c * aqr;
      }
      for (int r = 0; r < 3; ++r) {
        const double vrp = v[r][p], vrq = v[r][q];
        v[r][p] = c * vrp - s * vrq;
        v[r][q] = s * vrp + c * vrq;
      }
    }
  }
  for (int k = 0; k < 3; ++k) lam[k] = a[k][k];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) V[3 * r + c] = v[r][c];
}

/* One GICP evaluation at (R, t): F = 1/2 sum rho(|r_i|^2) with Huber(0.5)
 * (align_gicp.cpp:70), r_i = C_i^{-1/2} (R s_i + t - d_i),
 * C_i = S_d + R S_s R^T (gicp_cost.hpp:50-69), and the Gauss-Newton
 * quantities of Ceres' robust corrector for a loss with rho'' <= 0
 * (J~ = sqrt(rho') J): H = sum rho' J^T J, g = sum rho' J^T r, J the exact
 * Jacobian w.r.t. (w, t), R(w) = exp([w]x) R, including the dependence of
 * C_i^{-1/2} on R (derivative of the inverse square root through the
 * eigen-decomposition).  H row-major 6x6. */
double orc_gicp_eval(const float* src, int64_t n, const float* dst, const float* src_covs,
                     const float* dst_covs, const int32_t* dst_idx, const double R[9],
                     const double t[3], double H[36], double g[6]) {
  double F = 0.0;
  if (H) memset(H, 0, sizeof(double) * 36);
  if (g) memset(g, 0, sizeof(double) * 6);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j = dst_idx[i];
    const float* Ss = src_covs + 9 * i; /* col-major (Eigen) = symmetric anyway */
    const float* Sd = dst_covs + 9 * j;
    double A[9], C[9], RS[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 3; ++k) s += R[3 * r + k] * (double)Ss[3 * c + k];
        RS[3 * r + c] = s;
      }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 3; ++k) s += RS[3 * r + k] * R[3 * c + k];
        A[3 * r + c] = s;
      }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) C[3 * r + c] = (double)Sd[3 * c + r] + A[3 * r + c];
    /* symmetrise (rounding) */
    for (int r = 0; r < 3; ++r)
      for (int c = r + 1; c < 3; ++c) {
        const double m = 0.5 * (C[3 * r + c] + C[3 * c + r]);
        C[3 * r + c] = C[3 * c + r] = m;
      }
    double lam[3], V[9];
    gicp_sym_eig3(C, lam, V);
    double is[3];
    for (int k = 0; k < 3; ++k) is[k] = 1.0 / sqrt(lam[k] > 1e-30 ? lam[k] : 1e-30);
    double M[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int k = 0; k < 3; ++k) s += V[3 * r + k] * is[k] * V[3 * c + k];
        M[3 * r + c] = s;
      }
    double Rs[3], dl[3];
    for (int r = 0; r < 3; ++r) {
      Rs[r] = R[3 * r] * src[3 * i] + R[3 * r + 1] * src[3 * i + 1] + R[3 * r + 2] * src[3 * i + 2];
      dl[r] = Rs[r] + t[r] - (double)dst[3 * j + r];
    }
    double res[3];
    for (int r = 0; r < 3; ++r) res[r] = M[3 * r] * dl[0] + M[3 * r + 1] * dl[1] + M[3 * r + 2] * dl[2];
    const double s2 = res[0] * res[0] + res[1] * res[1] + res[2] * res[2];
    const double rho = s2 <= 0.25 ? s2 : sqrt(s2) - 0.25;
    const double rho1 = s2 <= 0.25 ? 1.0 : 0.5 / sqrt(s2);
    F += 0.5 * rho;
    if (!H) continue;
    /* Daleckii-Krein weights of X -> X^{-1/2} */
    double W[9];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        const double la = lam[a] > 1e-30 ? lam[a] : 1e-30, lb = lam[b] > 1e-30 ? lam[b] : 1e-30;
        W[3 * a + b] = fabs(la - lb) > 1e-12 * (la + lb) ? (is[a] - is[b]) / (la - lb)
                                                         : -0.5 * is[a] / la;
      }
    double J[3][6];
    for (int k = 0; k < 3; ++k) {
      /* E = G_k A - A G_k, G_k = [e_k]x */
      double G[9] = {0};
      if (k == 0) { G[5] = -1; G[7] = 1; }
      if (k == 1) { G[2] = 1; G[6] = -1; }
      if (k == 2) { G[1] = -1; G[3] = 1; }
      double E[9];
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          double s = 0;
          for (int q = 0; q < 3; ++q) s += G[3 * r + q] * A[3 * q + c] - A[3 * r + q] * G[3 * q + c];
          E[3 * r + c] = s;
        }
      double B[9], T[9], dM[9];
      for (int a = 0; a < 3; ++a) /* B = V^T E V */
        for (int b = 0; b < 3; ++b) {
          double s = 0;
          for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) s += V[3 * r + a] * E[3 * r + c] * V[3 * c + b];
          B[3 * a + b] = s * W[3 * a + b];
        }
      for (int r = 0; r < 3; ++r) /* dM = V B V^T */
        for (int b = 0; b < 3; ++b) {
          double s = 0;
          for (int a = 0; a < 3; ++a) s += V[3 * r + a] * B[3 * a + b];
          T[3 * r + b] = s;
        }
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
          double s = 0;
          for (int b = 0; b < 3; ++b) s += T[3 * r + b] * V[3 * c + b];
          dM[3 * r + c] = s;
        }
      /* d(delta)/dw_k = e_k x (R s) */
      double ex[3] = {0, 0, 0};
      if (k == 0) { ex[1] = -Rs[2]; ex[2] = Rs[1]; }
      if (k == 1) { ex[0] = Rs[2]; ex[2] = -Rs[0]; }
      if (k == 2) { ex[0] = -Rs[1]; ex[1] = Rs[0]; }
      for (int r = 0; r < 3; ++r)
        J[r][k] = dM[3 * r] * dl[0] + dM[3 * r + 1] * dl[1] + dM[3 * r + 2] * dl[2] +
                  M[3 * r] * ex[0] + M[3 * r + 1] * ex[1] + M[3 * r + 2] * ex[2];
    }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) J[r][3 + c] = M[3 * r + c];
    for (int a = 0; a < 6; ++a) {
      double ga = 0;
      for (int r = 0; r < 3; ++r) ga += J[r][a] * res[r];
      g[a] += rho1 * ga;
      for (int b = 0; b < 6; ++b) {
        double h = 0;
        for (int r = 0; r < 3; ++r) h += J[r][a] * J[r][b];
        H[6 * a + b] += rho1 * h;
      }
    }
  }
  return F;
}

static void gicp_rodrigues(const double w[3], double E[9]) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const double th = sqrt(th2);
  double a, b;
  if (th < 1e-8) {
    a = 1.0 - th2 / 6.0;
    b = 0.5 - th2 / 24.0;
  } else {
    a = sin(th) / th;
    b = (1.0 - cos(th)) / th2;
  }
  const double K[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      double kk = 0;
      for (int q = 0; q < 3; ++q) kk += K[3 * r + q] * K[3 * q + c];
      E[3 * r + c] = (r == c ? 1.0 : 0.0) + a * K[3 * r + c] + b * kk;
    }
}

/* (H + lambda diag(H)) x = -g by Cholesky; 0 when not positive definite */
static int gicp_lm_step(const double H[36], const double g[6], double lambda, double x[6]) {
  double L[36];
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b) L[6 * a + b] = H[6 * a + b] + (a == b ? lambda * H[6 * a + a] : 0.0);
  for (int j = 0; j < 6; ++j) {
    double s = L[6 * j + j];
    for (int k = 0; k < j; ++k) s -= L[6 * j + k] * L[6 * j + k];
    if (!(s > 0)) return 0;
    L[6 * j + j] = sqrt(s);
    for (int i = j + 1; i < 6; ++i) {
      double u = L[6 * i + j];
      for (int k = 0; k < j; ++k) u -= L[6 * i + k] * L[6 * j + k];
      L[6 * i + j] = u / L[6 * j + j];
    }
  }
  double y[6];
  for (int i = 0; i < 6; ++i) {
    double s = -g[i];
    for (int k = 0; k < i; ++k) s -= L[6 * i + k] * y[k];
    y[i] = s / L[6 * i + i];
  }
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < 6; ++k) s -= L[6 * k + i] * x[k];
    x[i] = s / L[6 * i + i];
  }
  return 1;
}

/* ComputeAlignment with given covariances and correspondences
 * (align_gicp.cpp:41-103): Ceres' Levenberg-Marquardt restated as the
 * build's own LM (DESIGN.md "GICP"): evaluate the candidate; accept when F
 * drops (lambda /= 3, floor 1e-12) else lambda *= 4; stop when the step norm
 * < 1e-10, the relative drop of an accepted step < 1e-6 (Ceres'
 * Solver::Options::function_tolerance default: GetOptions(), align_gicp.cpp:13-37,
 * sets no tolerance), lambda > 1e10, or after max_iter evaluations.  Returns the final F (Ceres' final_cost); pose_out 4x4
 * col-major float (R from the fp64 rotation, as q.toRotationMatrix()). */
#define ORC_GICP_FTOL 1e-6 /* Ceres' default function_tolerance */
double orc_gicp_solve(const float* src, int64_t n, const float* dst, const float* src_covs,
                      const float* dst_covs, const int32_t* dst_idx, const float seed[16],
                      int max_iter, float pose_out[16], int* iters_out) {
  double R[9], t[3];
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) R[3 * r + c] = seed[4 * c + r];
    t[r] = seed[12 + r];
  }
  double H[36], g[6];
  double F = orc_gicp_eval(src, n, dst, src_covs, dst_covs, dst_idx, R, t, H, g);
  double lambda = 1e-4;
  int it = 1;
  while (it < max_iter) {
    double x[6] = {0, 0, 0, 0, 0, 0};
    if (!gicp_lm_step(H, g, lambda, x)) {
      lambda *= 4.0;
      if (lambda > 1e10) break;
      continue;
    }
    const double nx = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3] + x[4] * x[4] + x[5] * x[5]);
    if (nx < 1e-10) break;
    double E[9], R2[9], t2[3];
    gicp_rodrigues(x, E);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int q = 0; q < 3; ++q) s += E[3 * r + q] * R[3 * q + c];
        R2[3 * r + c] = s;
      }
    for (int r = 0; r < 3; ++r) t2[r] = t[r] + x[3 + r];
    double H2[36], g2[6];
    const double F2 = orc_gicp_eval(src, n, dst, src_covs, dst_covs, dst_idx, R2, t2, H2, g2);
    ++it;
    if (F2 < F) {
      const double drop = (F - F2) / (F > 0 ? F : 1.0);
      memcpy(R, R2, sizeof(R));
      memcpy(t, t2, sizeof(t));
      memcpy(H, H2, sizeof(H));
      memcpy(g, g2, sizeof(g));
      F = F2;
      lambda = lambda / 3.0 > 1e-12 ? lambda / 3.0 : 1e-12;
      if (drop < ORC_GICP_FTOL) break;
    } else {
      lambda *= 4.0;
      if (lambda > 1e10) break;
    }
  }
  for (int c = 0; c < 3; ++c) {
    for (int r = 0; r < 3; ++r) pose_out[4 * c + r] = (float)R[3 * r + c];
    pose_out[4 * c + 3] = 0.f;
  }
  for (int r = 0; r < 3; ++r) pose_out[12 + r] = (float)t[r];
  pose_out[15] = 1.f;
  if (iters_out) *iters_out = it;
  return F;
}

/* ComputeAlignment(src, dst, &T) (align_gicp.cpp:105-163): covariances of
 * both clouds (k = 32, use_gicp = false), estimate = Identity (the
 * reference ignores T's value), 16 x { correspondences = exact 1-NN of
 * estimate * src in dst; estimate = LM solve seeded at estimate }.  Returns
 * the last solve's cost; T = estimate. */
double orc_gicp_align(const float* src, int64_t n, const float* dst, int64_t m,
                      int outer_iters, int max_inner, float pose_out[16]) {
  orc_kdtree* ts = orc_kdtree_build(src, n, 16);
  orc_kdtree* td = orc_kdtree_build(dst, m, 16);
  float* cs = (float*)malloc(sizeof(float) * 9 * (size_t)n);
  float* cd = (float*)malloc(sizeof(float) * 9 * (size_t)m);
  orc_compute_covariances(src, n, ts, 0, cs);
  orc_compute_covariances(dst, m, td, 0, cd);
  float est[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  float* tmp = (float*)malloc(sizeof(float) * 3 * (size_t)n);
  int32_t* nn = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  double cost = 0.0;
  for (int o = 0; o < outer_iters; ++o) {
    orc_transform_points(est, src, n, tmp);
    for (int64_t i = 0; i < n; ++i) {
      float d2;
      orc_kdtree_knn(td, tmp + 3 * i, 1, nn + i, &d2);
    }
    float next[16];
    cost = orc_gicp_solve(src, n, dst, cs, cd, nn, est, max_inner, next, NULL);
    memcpy(est, next, sizeof(est));
  }
  memcpy(pose_out, est, sizeof(est));
  free(cs);
  free(cd);
  free(tmp);
  free(nn);
  orc_kdtree_free(ts);
  orc_kdtree_free(td);
  return cost;
}

/* ==== f4: CloudAccumulator (rs_replay_app.cpp:76-129) ======================== */
struct orc_accum {
  float inv;
  int64_t cap, used, count, list_cap;
  int32_t* keys; /* 3 per slot */
  uint8_t* used_flag;
  float* list;
};

static int orc_trunc_key(float x, float inv) {
  const float q = x * inv;
  return (q >= -2147483648.0f && q < 2147483648.0f) ? (int)q : INT_MIN;
}

orc_accum* orc_accum_create(float voxel_size) {
  orc_accum* a = (orc_accum*)calloc(1, sizeof(orc_accum));
  a->inv = (float)(1.0 / (double)voxel_size); /* :91-92 */
  return a;
}

void orc_accum_free(orc_accum* a) {
  if (!a) return;
  free(a->keys);
  free(a->used_flag);
  free(a->list);
  free(a);
}

static uint64_t orc_key_hash(int x, int y, int z) {
  uint64_t h = ((uint64_t)(uint32_t)x * 73856093u) ^ ((uint64_t)(uint32_t)y * 19349663u) ^
               ((uint64_t)(uint32_t)z * 83492791u);
  return h ^ (h >> 17);
}

static void orc_accum_rehash(orc_accum* a, int64_t need) {
  int64_t cap = a->cap ? a->cap : 1024;
  while (cap < 2 * need) cap <<= 1;
  if (cap == a->cap) return;
  free(a->keys);
  free(a->used_flag);
  a->keys = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)cap);
  a->used_flag = (uint8_t*)calloc((size_t)cap, 1);
  a->cap = cap;
  for (int64_t j = 0; j < a->count; ++j) {
    const float* p = a->list + 3 * j;
    const int k0 = orc_trunc_key(p[0], a->inv), k1 = orc_trunc_key(p[1], a->inv),
              k2 = orc_trunc_key(p[2], a->inv);
    int64_t s = (int64_t)(orc_key_hash(k0, k1, k2) & (uint64_t)(cap - 1));
    while (a->used_flag[s]) s = (s + 1) & (cap - 1);
    a->used_flag[s] = 1;
    a->keys[3 * s] = k0;
    a->keys[3 * s + 1] = k1;
    a->keys[3 * s + 2] = k2;
  }
}

/* AddCloud (:95-106): p = xfm * point (:98), key = (p * inv).cast<int>()
 * (:108-110), emplace only when new */
void orc_accum_add(orc_accum* a, const float pose[16], const float* xyz, int64_t n) {
  orc_accum_rehash(a, a->count + n);
  if (a->list_cap < a->count + n) {
    int64_t c = a->list_cap ? a->list_cap : 1024;
    while (c < a->count + n) c *= 2;
    a->list = (float*)realloc(a->list, sizeof(float) * 3 * (size_t)c);
    a->list_cap = c;
  }
  for (int64_t i = 0; i < n; ++i) {
    float p[3];
    orc_transform_points(pose, xyz + 3 * i, 1, p);
    const int k0 = orc_trunc_key(p[0], a->inv), k1 = orc_trunc_key(p[1], a->inv),
              k2 = orc_trunc_key(p[2], a->inv);
    int64_t s = (int64_t)(orc_key_hash(k0, k1, k2) & (uint64_t)(a->cap - 1));
    int found = 0;
    while (a->used_flag[s]) {
      if (a->keys[3 * s] == k0 && a->keys[3 * s + 1] == k1 && a->keys[3 * s + 2] == k2) {
        found = 1;
        break;
      }
      s = (s + 1) & (a->cap - 1);
    }
    if (found) continue;
    a->used_flag[s] = 1;
    a->keys[3 * s] = k0;
    a->keys[3 * s + 1] = k1;
    a->keys[3 * s + 2] = k2;
    memcpy(a->list + 3 * a->count, p, sizeof(p));
    ++a->count;
  }
}

/* ExtractPointCloud (:112-121), insertion order; returns the count */
int64_t orc_accum_extract(const orc_accum* a, float* out) {
  if (out && a->count) memcpy(out, a->list, sizeof(float) * 3 * (size_t)a->count);
  return a->count;
}
