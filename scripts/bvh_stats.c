// CPU replay of the GPU BVH build + stackless traversal to count node visits
// (diagnostic only).  Build: gcc -O2 -o /tmp/bvh_stats bvh_stats.c -lm
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef struct { float x, y, z, w; } f4;
static uint32_t spread10(uint32_t v) {
  v &= 0x3ff; v = (v | (v << 16)) & 0x030000FF; v = (v | (v << 8)) & 0x0300F00F;
  v = (v | (v << 4)) & 0x030C30C3; v = (v | (v << 2)) & 0x09249249; return v; }
static uint32_t *gkeys;
static int cmp(const void* a, const void* b) {
  uint32_t ka = gkeys[*(const int*)a], kb = gkeys[*(const int*)b];
  if (ka != kb) return ka < kb ? -1 : 1; return *(const int*)a - *(const int*)b; }
int main(int argc, char** argv) {
  // reads float32 xyz: target file, query file
  FILE* f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long m = ftell(f) / 12; fseek(f, 0, SEEK_SET);
  float* dst = malloc(m * 12); fread(dst, 12, m, f); fclose(f);
  f = fopen(argv[2], "rb"); fseek(f, 0, SEEK_END); long n = ftell(f) / 12; fseek(f, 0, SEEK_SET);
  float* q = malloc(n * 12); fread(q, 12, n, f); fclose(f);
  int leafsz = argc > 3 ? atoi(argv[3]) : 16;
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (long i = 0; i < m; ++i) for (int d = 0; d < 3; ++d) { lo[d] = fminf(lo[d], dst[3*i+d]); hi[d] = fmaxf(hi[d], dst[3*i+d]); }
  float ext = fmaxf(fmaxf(hi[0]-lo[0], hi[1]-lo[1]), hi[2]-lo[2]); float sc = 1023.f / ext;
  gkeys = malloc(m * 4); int* perm = malloc(m * 4);
  for (long i = 0; i < m; ++i) { uint32_t c[3]; for (int d = 0; d < 3; ++d) c[d] = (uint32_t)fminf(fmaxf((dst[3*i+d]-lo[d])*sc, 0), 1023);
    gkeys[i] = (spread10(c[0]) << 2) | (spread10(c[1]) << 1) | spread10(c[2]); perm[i] = i; }
  qsort(perm, m, 4, cmp);
  f4* pts = malloc(m * 16); for (long i = 0; i < m; ++i) { int j = perm[i]; pts[i].x = dst[3*j]; pts[i].y = dst[3*j+1]; pts[i].z = dst[3*j+2]; memcpy(&pts[i].w, &j, 4); }
  long nl = 1; while (nl * leafsz < m) nl <<= 1;
  int* ls = malloc((nl + 1) * 4); for (long L = 0; L <= nl; ++L) ls[L] = (int)(L * m / nl);
  f4* nodes = malloc(4 * nl * 16);
  for (long L = 0; L < nl; ++L) { f4 l = {INFINITY, INFINITY, INFINITY, 0}, h = {-INFINITY, -INFINITY, -INFINITY, 0};
    for (int i = ls[L]; i < ls[L+1]; ++i) { l.x = fminf(l.x, pts[i].x); l.y = fminf(l.y, pts[i].y); l.z = fminf(l.z, pts[i].z);
      h.x = fmaxf(h.x, pts[i].x); h.y = fmaxf(h.y, pts[i].y); h.z = fmaxf(h.z, pts[i].z); }
    nodes[2*(nl+L)] = l; nodes[2*(nl+L)+1] = h; }
  for (long k = nl - 1; k >= 1; --k) {
    f4 l0 = nodes[4*k], h0 = nodes[4*k+1], l1 = nodes[4*k+2], h1 = nodes[4*k+3], l, h;
    l.x = fminf(l0.x, l1.x); l.y = fminf(l0.y, l1.y); l.z = fminf(l0.z, l1.z); h.x = fmaxf(h0.x, h1.x); h.y = fmaxf(h0.y, h1.y); h.z = fmaxf(h0.z, h1.z);
    int e0 = !(l0.x <= h0.x), e1 = !(l1.x <= h1.x); float split; int ab;
    if (e0 || e1) { ab = 0; split = e1 ? INFINITY : -INFINITY; } else {
      float c0[3] = {.5f*(l0.x+h0.x), .5f*(l0.y+h0.y), .5f*(l0.z+h0.z)}, c1[3] = {.5f*(l1.x+h1.x), .5f*(l1.y+h1.y), .5f*(l1.z+h1.z)};
      int ax = 0; float b = fabsf(c1[0]-c0[0]); for (int a = 1; a < 3; ++a) if (fabsf(c1[a]-c0[a]) > b) { b = fabsf(c1[a]-c0[a]); ax = a; }
      split = .5f * (c0[ax] + c1[ax]); ab = ax | (c0[ax] <= c1[ax] ? 0 : 4); }
    l.w = split; memcpy(&h.w, &ab, 4); nodes[2*k] = l; nodes[2*k+1] = h; }
  // traversal stats
  long tot_steps = 0, tot_leaves = 0, tot_pts = 0, maxsteps = 0; double sumd = 0;
  long hist[8] = {0};
  for (long i = 0; i < n; ++i) {
    float qx = q[3*i], qy = q[3*i+1], qz = q[3*i+2]; float bd2 = FLT_MAX; int bid = 0; long steps = 0, leaves = 0, np_ = 0;
    int cur = 1, prev = 0;
    while (cur) { int parent = cur >> 1; f4 l = nodes[2*cur], h = nodes[2*cur+1]; int next; ++steps;
      if (prev == parent) {
        float ex = fmaxf(fmaxf(l.x - qx, qx - h.x), 0), ey = fmaxf(fmaxf(l.y - qy, qy - h.y), 0), ez = fmaxf(fmaxf(l.z - qz, qz - h.z), 0);
        float bd = ex*ex + ey*ey + ez*ez;
        if (bd > bd2) next = parent;
        else if (cur >= nl) { int L = cur - nl; ++leaves; for (int p = ls[L]; p < ls[L+1]; ++p) { ++np_; float dx = qx - pts[p].x, dy = qy - pts[p].y, dz = qz - pts[p].z;
            float d2 = dx*dx; d2 += dy*dy; d2 += dz*dz; int id; memcpy(&id, &pts[p].w, 4); if (d2 < bd2 || (d2 == bd2 && id < bid)) { bd2 = d2; bid = id; } } next = parent; }
        else { int abx; memcpy(&abx, &h.w, 4); int ax = abx & 3; float qa = ax == 0 ? qx : ax == 1 ? qy : qz; int ql = qa < l.w; int ll = (abx & 4) == 0; next = (ql == ll) ? 2*cur : 2*cur+1; }
      } else { int abx; memcpy(&abx, &h.w, 4); int ax = abx & 3; float qa = ax == 0 ? qx : ax == 1 ? qy : qz; int ql = qa < l.w; int ll = (abx & 4) == 0; int nc = (ql == ll) ? 2*cur : 2*cur+1;
        next = (prev == nc) ? (prev ^ 1) : parent; }
      prev = cur; cur = next; }
    tot_steps += steps; tot_leaves += leaves; tot_pts += np_; if (steps > maxsteps) maxsteps = steps; sumd += sqrt(bd2);
    int b = steps < 64 ? 0 : steps < 128 ? 1 : steps < 256 ? 2 : steps < 512 ? 3 : steps < 1024 ? 4 : steps < 4096 ? 5 : 6; hist[b]++;
  }
  printf("m=%ld n=%ld nleaves=%ld avg steps %.1f leaves %.1f pts %.1f max steps %ld mean dist %.4f\n", m, n, nl, (double)tot_steps/n, (double)tot_leaves/n, (double)tot_pts/n, maxsteps, sumd/n);
  printf("steps hist <64:%ld <128:%ld <256:%ld <512:%ld <1k:%ld <4k:%ld >=4k:%ld\n", hist[0], hist[1], hist[2], hist[3], hist[4], hist[5], hist[6]);
  return 0; }
