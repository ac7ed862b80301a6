/* ASan/UBSan driver for the CPU oracle (test infrastructure; SURVEY.md §5:
 * sanitizers on host code).  Built by `make -C oracle asan` with
 * -fsanitize=address,undefined -fno-sanitize-recover=all and run by
 * tests/test_oracle_sanitizers.py: every entry point of rst_oracle.h on a
 * seeded synthetic depth frame (unprojection, kd-tree, NN, normals, ICP in
 * both sum modes, point-to-plane, RemoveNans / DownsampleVoxel with NaNs,
 * GICP, FPFH, matches, the map accumulator) plus the edge sizes the tests
 * use (0-3 points).  Exit status 0 = no sanitizer report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rst_oracle.h"

static uint32_t rng = 12345u;
static float frand(void) {
  rng = rng * 1664525u + 1013904223u;
  return (float)(rng >> 8) / (float)(1u << 24);
}

/* a tilted plane plus a bump, rendered as u16 depth in mm */
static void make_depth(uint16_t* d, int w, int h, float tilt) {
  for (int v = 0; v < h; ++v)
    for (int u = 0; u < w; ++u) {
      const float x = (u - w / 2) / (float)w, y = (v - h / 2) / (float)h;
      float z = 1.5f + tilt * x + 0.3f * expf(-20.f * (x * x + y * y)) + 0.001f * frand();
      d[v * w + u] = (frand() < 0.03f) ? 0 : (uint16_t)(z * 1000.f);
    }
}

int main(void) {
  const int w = 96, h = 72;
  const float K[4] = {60.f, 60.f, w / 2.f, h / 2.f};
  uint16_t* da = malloc(sizeof(uint16_t) * w * h);
  uint16_t* db = malloc(sizeof(uint16_t) * w * h);
  make_depth(da, w, h, 0.2f);
  make_depth(db, w, h, 0.21f);
  float* pa = malloc(sizeof(float) * 3 * w * h);
  float* pb = malloc(sizeof(float) * 3 * w * h);
  const int64_t m = orc_unproject(da, w, h, K, 0.001f, 0, pa);
  const int64_t n = orc_unproject(db, w, h, K, 0.001f, 0, pb);
  float* tmp = malloc(sizeof(float) * 3 * w * h);
  orc_unproject(da, w, h, K, 0.001f, 1, tmp);
  orc_unproject_strided(da, w, h, 2, K, 0.001f, 0, tmp);
  const float vp[3] = {0.f, 0.f, 0.f};
  float* gn = malloc(sizeof(float) * 3 * w * h);
  orc_grid_normals(da, w, h, 1, K, 0.001f, 2, vp, gn);

  orc_kdtree* t = orc_kdtree_build(pa, m, 16);
  int32_t* idx = malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1) * 33);
  float* d2 = malloc(sizeof(float) * (size_t)(n > 0 ? n : 1) * 33);
  orc_nn_batch(t, pb, n, idx, d2);
  orc_nn_bruteforce(pa, m, pb, 64, idx, d2);
  orc_kdtree_knn(t, pb, 16, idx, d2);
  float* nrm = malloc(sizeof(float) * 3 * (size_t)m);
  orc_compute_normals(pa, m, t, 16, vp, nrm);

  for (int mode = 0; mode < 2; ++mode) {
    float T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    float mc = 0.f;
    orc_icp_trace tr;
    memset(&tr, 0, sizeof(tr));
    orc_align_icp_ex(pb, n, pa, m, t, 16, T, &mc, &tr, mode);
  }
  {
    float T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    orc_align_icp(pb, n, pa, m, NULL, 4, T, NULL, NULL);
    float Tp[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    float mc = 0.f;
    orc_align_p2plane(pb, n, pa, nrm, m, t, 10, 1e-6f, 1.f, 0.f, Tp, &mc);
    const float sm[3] = {0.f, 0.f, 1.5f};
    double part[16];
    orc_p2point_partials(pb, n, t, pa, T, sm, 1.f, part);
    float c3[3];
    orc_centroid(pb, n, c3);
  }
  /* edge sizes: the early-false paths and 1-3 point targets */
  for (int k = 0; k <= 3; ++k) {
    float T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    orc_align_icp(pb, k, pa, k, NULL, 4, T, NULL, NULL);
    if (k > 0) {
      orc_kdtree* tk = orc_kdtree_build(pa, k, 16);
      orc_nn_batch(tk, pb, 16, idx, d2);
      orc_kdtree_free(tk);
    }
  }
  /* RemoveNans / DownsampleVoxel with non-finite and out-of-range points */
  {
    const int64_t q = 256;
    float* c = malloc(sizeof(float) * 3 * q);
    for (int64_t i = 0; i < 3 * q; ++i) c[i] = (frand() - 0.5f) * 4.f;
    c[3] = NAN;
    c[10] = INFINITY;
    c[20] = -INFINITY;
    c[30] = 3e38f;
    float* o = malloc(sizeof(float) * 3 * (size_t)(m > q ? m : q));
    orc_remove_nans(c, q, o);
    orc_downsample_voxel(c, q, 0.05f, o);
    orc_downsample_voxel(pa, m, 0.02f, o);
    free(c);
    free(o);
  }
  /* GICP, FPFH, matches on a downsampled pair */
  {
    float* sa = malloc(sizeof(float) * 3 * (size_t)m);
    float* sb = malloc(sizeof(float) * 3 * (size_t)n);
    const int64_t ma = orc_downsample_voxel(pa, m, 0.05f, sa);
    const int64_t nb = orc_downsample_voxel(pb, n, 0.05f, sb);
    float Tg[16];
    orc_gicp_align(sb, nb, sa, ma, 2, 8, Tg);
    float* fa = malloc(sizeof(float) * 33 * (size_t)ma);
    float* fb = malloc(sizeof(float) * 33 * (size_t)nb);
    orc_compute_fpfh(sa, ma, vp, 16, 0.15f, fa);
    orc_compute_fpfh(sb, nb, vp, 16, 0.15f, fb);
    orc_compute_matches(fb, nb, fa, ma, 2, idx, d2);
    orc_accum* acc = orc_accum_create(0.05f);
    orc_accum_add(acc, Tg, sa, ma);
    orc_accum_add(acc, Tg, sb, nb);
    float* out = malloc(sizeof(float) * 3 * (size_t)(ma + nb));
    orc_accum_extract(acc, out);
    orc_accum_free(acc);
    free(out);
    free(fa);
    free(fb);
    free(sa);
    free(sb);
  }
  orc_kdtree_free(t);
  free(nrm);
  free(idx);
  free(d2);
  free(gn);
  free(tmp);
  free(pa);
  free(pb);
  free(da);
  free(db);
  printf("oracle sanitizer run ok: n=%lld m=%lld\n", (long long)n, (long long)m);
  return 0;
}
