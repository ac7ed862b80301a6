// bvh_selftest.cpp -- CPU check of the exact searches in rst_bvh.hpp.
//
// The product runs these searches on the GPU; they are written
// __host__ __device__, so the very same code is exercised here on the CPU
// against brute force (lexicographic (d2, index) minimum, the contract of
// rst_target_query_nn).  A CPU build of the index mirrors build.hip's
// pipeline (Morton order, fixed-size leaves, make_leaf / make_internal).
//
// Usage: bvh_selftest [seed]   -- exit 0 on success, prints a summary.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "rst_bvh.hpp"
#include "rst_wave_nn.hpp"

using namespace rst;

namespace {

void check(bool ok, const char* what, int m, int q);

struct Index {
  std::vector<float4> pts;
  std::vector<uint32_t> codes;
  std::vector<int32_t> lstart, pleaf;
  std::vector<float4> nodes;
  std::vector<float4> adj, adj2, adj3;
  std::vector<float> reach, reach2, reach3;
  BvhView bv;
  AdjView av;
};

Index build(const std::vector<float>& xyz) {
  Index ix;
  const int m = (int)(xyz.size() / 3);
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = 0; i < m; ++i)
    if (finite3(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]))
      for (int d = 0; d < 3; ++d) {
        lo[d] = std::min(lo[d], xyz[3 * i + d]);
        hi[d] = std::max(hi[d], xyz[3 * i + d]);
      }
  const float ext = std::max(std::max(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]);
  const float sc = ext > 0 ? 1023.0f / ext : 0.0f;
  std::vector<std::pair<uint32_t, int>> kv(m);
  for (int i = 0; i < m; ++i) {
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    uint32_t code = 0x3fffffffu;
    if (finite3(x, y, z)) {
      auto q = [&](float v, float l) { return (uint32_t)std::min(std::max((v - l) * sc, 0.0f), 1023.0f); };
      code = (spread10(q(x, lo[0])) << 2) | (spread10(q(y, lo[1])) << 1) | spread10(q(z, lo[2]));
    }
    kv[i] = {code, i};
  }
  std::stable_sort(kv.begin(), kv.end(),
                   [](const auto& a, const auto& b) { return a.first < b.first; });
  ix.pts.resize(std::max(m, 1) + kPtsPad);
  ix.codes.resize(std::max(m, 1));
  for (int i = 0; i < m; ++i) {
    const int j = kv[i].second;
    ix.pts[i] = make_float4(xyz[3 * j], xyz[3 * j + 1], xyz[3 * j + 2], i2f(j));
    ix.codes[i] = kv[i].first;
  }
  // compact leaves (rst_bvh.hpp leaf_cut)
  ix.pleaf.assign(std::max(m, 1), 0);
  ix.lstart.clear();
  int seg = 0;
  for (int i = 0; i < m; ++i) {
    if (i == 0 || (ix.codes[i] >> kLeafCellShift) != (ix.codes[i - 1] >> kLeafCellShift)) seg = i;
    if (leaf_cut(ix.codes.data(), i, seg)) ix.lstart.push_back(i);
    ix.pleaf[i] = (int)ix.lstart.size() - 1;
  }
  const int NL = std::max((int)ix.lstart.size(), 1);
  int nl = 1, lg = 0;
  while (nl < NL) {
    nl <<= 1;
    ++lg;
  }
  while ((int)ix.lstart.size() <= nl) ix.lstart.push_back(m);
  ix.nodes.resize(4 * (size_t)nl);
  ix.bv.codes = ix.codes.data();
  ix.bv.bbox = nullptr;
  ix.bv.lstart = ix.lstart.data();
  ix.bv.pleaf = ix.pleaf.data();
  ix.bv.pts = ix.pts.data();
  ix.bv.nodes = ix.nodes.data();
  ix.bv.m = m;
  ix.bv.nleaves = nl;
  ix.bv.lg = lg;
  ix.bv.pad = 0;
  for (int L = 0; L < nl; ++L) make_leaf(ix.bv, ix.nodes.data(), L);
  for (int k = nl - 1; k >= 1; --k) make_internal(ix.nodes.data(), k);
  ix.adj.resize((size_t)nl * kAdjK * 2);
  ix.reach.resize(nl);
  if (m > 0)
    for (int L = 0; L < nl; ++L) {
      BestK<kAdjK + 1> r;
      r.init();
      leaf_knn(ix.bv, nl, L, r);
      adj_store(ix.bv, nl, r, L, ix.adj.data(), ix.reach.data());
    }
  const int n2 = std::max(nl >> kAdj2Shift, 1);
  ix.adj2.resize((size_t)n2 * kAdjK * 2);
  ix.reach2.assign(n2, 0.0f);
  if (m > 0 && nl >= (1 << kAdj2Shift))
    for (int L = 0; L < n2; ++L) {
      BestK<kAdjK + 1> r;
      r.init();
      leaf_knn(ix.bv, n2, L, r);
      adj_store(ix.bv, n2, r, L, ix.adj2.data(), ix.reach2.data());
    }
  const int n3 = std::max(nl >> kAdj3Shift, 1);
  ix.adj3.resize((size_t)n3 * kAdjK * 2);
  ix.reach3.assign(n3, 0.0f);
  if (m > 0 && nl >= (1 << kAdj3Shift))
    for (int L = 0; L < n3; ++L) {
      BestK<kAdjK + 1> r;
      r.init();
      leaf_knn(ix.bv, n3, L, r);
      adj_store(ix.bv, n3, r, L, ix.adj3.data(), ix.reach3.data());
    }
  ix.av.ent3 = ix.adj3.data();
  ix.av.reach3 = ix.reach3.data();
  ix.av.ent = ix.adj.data();
  ix.av.reach = ix.reach.data();
  ix.av.ent2 = ix.adj2.data();
  ix.av.reach2 = ix.reach2.data();
  return ix;
}

// leaf_knn against brute force over all leaf boxes
void check_adjacency(const Index& ix) {
  const int nl = ix.bv.nleaves;
  if (ix.bv.m <= 0) return;
  for (int L = 0; L < nl; L += std::max(1, nl / 64)) {
    std::vector<float> d;
    for (int X = 0; X < nl; ++X) {
      const float b = bbd2(ix.nodes[2 * (nl + L)], ix.nodes[2 * (nl + L) + 1],
                           ix.nodes[2 * (nl + X)], ix.nodes[2 * (nl + X) + 1]);
      if (b < FLT_MAX) d.push_back(b);
    }
    std::sort(d.begin(), d.end());
    bool ok = true;
    for (int j = 0; j < kAdjK; ++j) {
      const float4 a = ix.adj[((size_t)L * kAdjK + j) * 2];
      const float want = j < (int)d.size() ? sqrtf(d[j]) : INFINITY;
      ok &= a.w == want;
    }
    ok &= ix.reach[L] == (kAdjK < (int)d.size() ? sqrtf(d[kAdjK]) : INFINITY);
    check(ok, "adjacency", ix.bv.m, L);
  }
}

template <int K>
void brute(const std::vector<float>& xyz, float qx, float qy, float qz, BestK<K>& r) {
  r.init();
  if (!finite3(qx, qy, qz)) return;
  const int m = (int)(xyz.size() / 3);
  for (int j = 0; j < m; ++j)
    r.offer(d2_ref(qx, qy, qz, xyz[3 * j], xyz[3 * j + 1], xyz[3 * j + 2]), j, j);
}

int g_fail = 0;
long g_checks = 0;
long g_covered = 0, g_covered2 = 0, g_covered3 = 0, g_adj_tries = 0;
long g_wide = 0, g_knn_tries = 0, g_knn_cov = 0, g_list_tries = 0, g_list_holds = 0;

void check(bool ok, const char* what, int m, int q) {
  ++g_checks;
  if (!ok && g_fail++ < 20) fprintf(stderr, "FAIL %s m=%d query=%d\n", what, m, q);
}

// sorted position of original index j
int pos_of(const Index& ix, int j) {
  for (int i = 0; i < ix.bv.m; ++i)
    if (f2i(ix.pts[i].w) == j) return i;
  return -1;
}

void run_case(std::mt19937_64& rng, int m, int nq, int mode) {
  std::uniform_real_distribution<float> U(-1.0f, 1.0f);
  std::vector<float> xyz(3 * (size_t)m);
  for (int i = 0; i < m; ++i) {
    if (mode == 1) {  // coarse lattice: many exact ties and duplicates
      for (int d = 0; d < 3; ++d) xyz[3 * i + d] = std::floor(U(rng) * 4.0f) * 0.25f;
    } else if (mode == 2) {  // surface-like: a wavy sheet, dense
      const float u = U(rng), v = U(rng);
      xyz[3 * i] = u;
      xyz[3 * i + 1] = v;
      xyz[3 * i + 2] = 0.1f * std::sin(6.0f * u) * std::cos(5.0f * v) + 0.002f * U(rng);
    } else {
      for (int d = 0; d < 3; ++d) xyz[3 * i + d] = U(rng);
    }
  }
  if (mode == 3 && m > 4) {  // a few non-finite target points
    xyz[0] = NAN;
    xyz[4] = INFINITY;
  }
  const Index ix = build(xyz);
  check_adjacency(ix);
  std::uniform_int_distribution<int> P(0, std::max(m - 1, 0));
  for (int q = 0; q < nq; ++q) {
    float qx, qy, qz;
    if (q % 3 == 0 && m > 0) {  // near an existing point (tight searches)
      const int j = P(rng);
      qx = xyz[3 * j] + 0.01f * U(rng);
      qy = xyz[3 * j + 1] + 0.01f * U(rng);
      qz = xyz[3 * j + 2] + 0.01f * U(rng);
    } else {
      qx = 1.5f * U(rng);
      qy = 1.5f * U(rng);
      qz = 1.5f * U(rng);
    }
    if (q == 7) qx = NAN;
    BestK<1> b1;
    brute(xyz, qx, qy, qz, b1);
    BestK<4> b4;
    brute(xyz, qx, qy, qz, b4);
    // cold top-down
    Best1 r;
    r.init();
    search(ix.bv, -1, qx, qy, qz, r);
    check(r.d == b1.d[0] && (r.pos < 0 ? b1.pos[0] < 0 : r.id == b1.id[0]), "nn cold", m, q);
    // warm: from a random start, from the answer, seeded with the start's d2
    for (int w = 0; w < 2 && m > 0; ++w) {
      const int start = w == 0 ? P(rng) : (b1.pos[0] >= 0 ? pos_of(ix, b1.id[0]) : P(rng));
      Best1 s;
      s.init();
      const float4 p = ix.pts[start];
      if (finite3(qx, qy, qz)) s.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), start);
      Best1 s2 = s;
      search(ix.bv, start, qx, qy, qz, s);
      check(s.d == b1.d[0] && (s.pos < 0 ? b1.pos[0] < 0 : s.id == b1.id[0]), "nn warm", m, q);
      if (finite3(qx, qy, qz)) {
        search_from_fast(ix.bv, start, qx, qy, qz, s2);
        check(s2.d == b1.d[0] && (s2.pos < 0 ? b1.pos[0] < 0 : s2.id == b1.id[0]), "nn fast", m, q);
      }
      if (s.pos >= 0) check(f2i(ix.pts[s.pos].w) == s.id, "nn pos", m, q);
    }
    // adjacency search from a warm candidate near the answer
    if (m > 0 && finite3(qx, qy, qz)) {
      const int start = b1.pos[0] >= 0 && (q & 1) ? pos_of(ix, b1.id[0]) : P(rng);
      Best1 s;
      s.init();
      const float4 p = ix.pts[start];
      s.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), start);
      ++g_adj_tries;
      Best1 s2 = s;
      if (adj_search(ix.bv, ix.av, start, qx, qy, qz, s)) {
        ++g_covered;
        check(s.d == b1.d[0] && (s.pos < 0 ? b1.pos[0] < 0 : s.id == b1.id[0]), "adj", m, q);
      }
      Best1 s3 = s2;
      if (adj3_search(ix.bv, ix.av, start, qx, qy, qz, s3)) {
        ++g_covered3;
        check(s3.d == b1.d[0] && (s3.pos < 0 ? b1.pos[0] < 0 : s3.id == b1.id[0]), "adj3", m, q);
      }
      if (adj2_search(ix.bv, ix.av, start, qx, qy, qz, s2)) {
        ++g_covered2;
        check(s2.d == b1.d[0] && (s2.pos < 0 ? b1.pos[0] < 0 : s2.id == b1.id[0]), "adj2", m, q);
      }
    }
    // the ICP kernel's adjacency search (rst_wave_nn.hpp adj_search_wide)
    if (m > 0 && finite3(qx, qy, qz)) {
      const int start = b1.pos[0] >= 0 && (q & 2) ? pos_of(ix, b1.id[0]) : P(rng);
      Best1 s;
      s.init();
      const float4 p = ix.pts[start];
      s.offer(d2_ref(qx, qy, qz, p.x, p.y, p.z), f2i(p.w), start);
      if (adj_search_wide(ix.bv, ix.av, start, qx, qy, qz, s)) {
        ++g_wide;
        check(s.d == b1.d[0] && s.id == b1.id[0], "adj wide", m, q);
      }
    }
    // the ICP candidate lists: exact 8-NN through the adjacency, and a moved
    // query whose list certificate holds has its nearest neighbour on the list
    if (m > 0 && finite3(qx, qy, qz)) {
      const int start = b1.pos[0] >= 0 && (q & 4) ? pos_of(ix, b1.id[0]) : P(rng);
      BestK<8> k8;  // (no warm offer: the scan of start's own leaf offers it)
      k8.init();
      BestK<8> b8;
      brute(xyz, qx, qy, qz, b8);
      ++g_knn_tries;
      if (adj_knn_search(ix.bv, ix.av, start, qx, qy, qz, k8)) {
        ++g_knn_cov;
        bool ok = true;
        for (int j = 0; j < 8; ++j) ok &= k8.d[j] == b8.d[j] && (b8.pos[j] < 0 || k8.id[j] == b8.id[j]);
        check(ok, "adj knn", m, q);
        const float4 c = make_float4(qx, qy, qz, k8.d[7] < FLT_MAX ? k8.d[7] : -1.0f);
        for (int t = 0; t < 8; ++t) {
          const float sc = 1e-4f * powf(3.0f, (float)t);
          const float nx = qx + sc * U(rng), ny = qy + sc * U(rng), nz = qz + sc * U(rng);
          float dbest = FLT_MAX;
          int ibest = 0x7fffffff;
          for (int j = 0; j < 8; ++j) {
            if (k8.pos[j] < 0) continue;
            const float4 pj = ix.pts[k8.pos[j]];
            const float dj = d2_ref(nx, ny, nz, pj.x, pj.y, pj.z);
            if (lex_less(dj, f2i(pj.w), dbest, ibest)) {
              dbest = dj;
              ibest = f2i(pj.w);
            }
          }
          ++g_list_tries;
          if (list_cert_holds(c, dbest, nx, ny, nz)) {
            ++g_list_holds;
            BestK<1> bb;
            brute(xyz, nx, ny, nz, bb);
            check(bb.id[0] == ibest && bb.d[0] == dbest, "list cert", m, q);
          }
        }
      }
    }
    // k = 4, bottom-up from a random leaf
    if (m > 0) {
      BestK<4> k4;
      k4.init();
      search(ix.bv, P(rng), qx, qy, qz, k4);
      bool ok = true;
      for (int j = 0; j < 4; ++j) ok &= k4.d[j] == b4.d[j] && k4.id[j] == b4.id[j];
      check(ok, "knn4 warm", m, q);
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;
  std::mt19937_64 rng(seed);
  const int sizes[] = {0, 1, 2, 3, 7, 16, 17, 33, 100, 257, 1000, 4099, 20000};
  for (int m : sizes)
    for (int mode = 0; mode < 4; ++mode) run_case(rng, m, m >= 4099 ? 300 : 120, mode);
  printf("bvh_selftest: %ld checks, %d failures (adjacency covered %ld / level 2 %ld / level 3 "
         "%ld of %ld warm queries; wide %ld; 8-NN covered %ld of %ld; list certificates held %ld "
         "of %ld moves)\n", g_checks, g_fail, g_covered, g_covered2, g_covered3, g_adj_tries,
         g_wide, g_knn_cov, g_knn_tries, g_list_holds, g_list_tries);
  return g_fail == 0 ? 0 : 1;
}
