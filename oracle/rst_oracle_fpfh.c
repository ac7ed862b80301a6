/*
 * rst_oracle_fpfh.c -- CPU ORACLE for SURVEY.md §8f row f3 (FPFH global
 * initialisation).  TEST INFRASTRUCTURE ONLY, like rst_oracle.c: loaded by
 * tests/ only, never by the product.
 *
 * Restates rs_tracker/common/src/fpfh.cpp:20-165,248-300 with the kd-tree
 * replaced by brute-force radius lists in ascending index (the reference
 * visits them in nanoflann's traversal order: the SPFH bins are sums of one
 * repeated value, order-free; the FPFH weighted sums differ only in
 * rounding) and the 33-D distance of nanoflann's metric_L2
 * (L2_Adaptor::evalMetric: four dimensions per partial sum, then the rest).
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "rst_oracle.h"

#define ORC_BINS 11
#define ORC_F 33
#define ORC_PI 3.14159265358979323846 /* M_PI */

/* ComputePfh (fpfh.cpp:20-64), kSymmetricPfh; Vector3f dot / norm in Eigen's
 * unrolled redux order x0 + (x1 + x2), as mv_row (rst_oracle.c) */
static int orc_pfh(const float* p1, const float* n1, const float* p2, const float* n2,
                   float f[3]) {
  float dx = p2[0] - p1[0], dy = p2[1] - p1[1], dz = p2[2] - p1[2];
  const float distance = sqrtf(dx * dx + (dy * dy + dz * dz));
  if (distance == 0.0f) return 0;
  const float id = 1.0f / distance;
  dx = dx * id;
  dy = dy * id;
  dz = dz * id;
  const float n1_d = n1[0] * dx + (n1[1] * dy + n1[2] * dz);
  const float n2_d = n2[0] * dx + (n2[1] * dy + n2[2] * dz);
  float u_d, nt_d;
  if (fabsf(n1_d) < fabsf(n2_d)) {
    u_d = -n2_d;
    nt_d = -n1_d;
  } else {
    u_d = n1_d;
    nt_d = n2_d;
  }
  if (fabsf(u_d) >= 1.0f) return 0;
  const float v_norm = sqrtf(1.0f - u_d * u_d);
  const float n1n2 = n1[0] * n2[0] + (n1[1] * n2[1] + n1[2] * n2[2]);
  f[0] = atan2f(nt_d - n1n2 * u_d, n1n2 * v_norm);
  const float cx = n1[1] * n2[2] - n1[2] * n2[1];
  const float cy = n1[2] * n2[0] - n1[0] * n2[2];
  const float cz = n1[0] * n2[1] - n1[1] * n2[0];
  f[1] = (dx * cx + (dy * cy + dz * cz)) / v_norm;
  f[2] = u_d;
  return 1;
}

static int orc_pfh_bin(float f, float scale) {
  const int raw = (int)floor((double)ORC_BINS * ((double)(f * scale) + 0.5));
  return raw < 0 ? 0 : (raw > ORC_BINS - 1 ? ORC_BINS - 1 : raw);
}

static float orc_d2(const float* q, const float* p) {
  const float dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
  return (dx * dx + dy * dy) + dz * dz;
}

void orc_compute_fpfh(const float* xyz, int64_t n, const float viewpoint[3], int normal_k,
                      float radius, float* out) {
  orc_kdtree* t = orc_kdtree_build(xyz, n, 16);
  float* nrm = (float*)malloc(sizeof(float) * 3 * (size_t)(n > 0 ? n : 1));
  orc_compute_normals(xyz, n, t, normal_k, viewpoint, nrm); /* (:254-255) */
  orc_kdtree_free(t);
  const float r2 = radius * radius;
  const float s0 = (float)(1.0 / (2.0 * ORC_PI)); /* scale (:76) */
  float* spfh = (float*)calloc((size_t)(n > 0 ? n : 1) * ORC_F, sizeof(float));
  for (int64_t i = 0; i < n; ++i) { /* (:127-133) */
    int cnt = 0, h[ORC_F];
    memset(h, 0, sizeof(h));
    for (int64_t j = 0; j < n; ++j) {
      if (!(orc_d2(xyz + 3 * i, xyz + 3 * j) < r2)) continue;
      ++cnt;
      if (j == i) continue;
      float f[3];
      if (!orc_pfh(xyz + 3 * i, nrm + 3 * i, xyz + 3 * j, nrm + 3 * j, f)) continue;
      h[orc_pfh_bin(f[0], s0)] += 1;
      h[ORC_BINS + orc_pfh_bin(f[1], 0.5f)] += 1;
      h[2 * ORC_BINS + orc_pfh_bin(f[2], 0.5f)] += 1;
    }
    const float dhist = 1.0f / (float)(cnt - 1); /* (:78) */
    for (int b = 0; b < ORC_F; ++b) {
      float s = 0.0f;
      for (int c = 0; c < h[b]; ++c) s = s + dhist; /* (:91) */
      spfh[i * ORC_F + b] = s;
    }
  }
  for (int64_t i = 0; i < n; ++i) { /* (:136-163) */
    float feat[ORC_F];
    memset(feat, 0, sizeof(feat));
    for (int64_t j = 0; j < n; ++j) {
      const float d2 = orc_d2(xyz + 3 * i, xyz + 3 * j);
      if (!(d2 < r2) || j == i) continue;
      const float w = 1.0F / sqrtf(d2);
      for (int b = 0; b < ORC_F; ++b) feat[b] = feat[b] + w * spfh[j * ORC_F + b];
    }
    for (int k = 0; k < 3; ++k) {
      float s = 0.0f;
      for (int b = 0; b < ORC_BINS; ++b) s = s + feat[k * ORC_BINS + b];
      if (s > 0) {
        const float inv = 1.0f / s;
        for (int b = 0; b < ORC_BINS; ++b) feat[k * ORC_BINS + b] = feat[k * ORC_BINS + b] * inv;
      }
    }
    memcpy(out + i * ORC_F, feat, sizeof(feat));
  }
  free(spfh);
  free(nrm);
}

/* nanoflann metric_L2 in 33-D (L2_Adaptor::evalMetric) */
static float orc_feat_d2(const float* a, const float* b) {
  float r = 0.0f;
  for (int g = 0; g < 8; ++g) {
    const float d0 = a[4 * g] - b[4 * g], d1 = a[4 * g + 1] - b[4 * g + 1];
    const float d2 = a[4 * g + 2] - b[4 * g + 2], d3 = a[4 * g + 3] - b[4 * g + 3];
    r = r + (((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3);
  }
  const float d = a[32] - b[32];
  return r + d * d;
}

/* ComputeMatches (fpfh.cpp:285-300): exact k (1 or 2) nearest, ties to the
 * lower index */
void orc_compute_matches(const float* src, int64_t n, const float* dst, int64_t m, int k,
                         int32_t* idx, float* d2) {
  for (int64_t i = 0; i < n; ++i) {
    float b0 = FLT_MAX, b1 = FLT_MAX;
    int32_t i0 = 0, i1 = 0;
    int h0 = 0, h1 = 0;
    for (int64_t j = 0; j < m; ++j) {
      const float d = orc_feat_d2(src + i * ORC_F, dst + j * ORC_F);
      const int32_t jj = (int32_t)j;
      if (!h0 || d < b0 || (d == b0 && jj < i0)) {
        b1 = b0;
        i1 = i0;
        h1 = h0;
        b0 = d;
        i0 = jj;
        h0 = 1;
      } else if (!h1 || d < b1 || (d == b1 && jj < i1)) {
        b1 = d;
        i1 = jj;
        h1 = 1;
      }
    }
    idx[i * k] = i0;
    if (d2) d2[i * k] = b0;
    if (k > 1) {
      idx[i * k + 1] = h1 ? i1 : 0;
      if (d2) d2[i * k + 1] = h1 ? b1 : FLT_MAX;
    }
  }
}
