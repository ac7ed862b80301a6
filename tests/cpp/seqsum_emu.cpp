// Host emulation of seqsum.hip's kernels (test infrastructure): the same
// arithmetic (rst_seqsum.hpp) and the same indexing, one workgroup / lane
// after another, with bounds-checked containers.  It checks the map logic
// and every index bound on the CPU, bit for bit against the plain
// sequential float sum -- the GPU tests then check the kernels themselves.
//
//   seqsum_emu <in.f32> <n> <nch>   (in: n float4 rows)  ->  prints the sums
//                                     and the walk statistics per chain
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "rst_seqsum.hpp"

using namespace rst::sq;

namespace {

int nf_flags(float x) {
  if (std::isnan(x)) return 1;
  if (std::isinf(x)) return x > 0 ? 2 : 4;
  return 0;
}

float cand(float G, int e0, int r) { return (float)((double)G + std::ldexp((double)r, e0)); }

struct Chain {
  int64_t n;
  int nb, ng, nk;
  std::vector<float> x;
  std::vector<uint8_t> wflg;
  std::vector<double> ttot, inc, tinc;
  std::vector<int> bs, gs, ks;
  std::vector<Leaf> leaf;
  std::vector<GroupMap> grp;
  std::vector<SbMap> sbm;
  int stats[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int work[3] = {0, 0, 0};  // leaf maps, group maps, superblock maps built
  // a stretch of a longer chain (the sharded loop: seqsum.hip's p0 / s_in):
  // the fp64 prefix before it (the guesses' offset) and the chain's value
  // where it starts (the walk's start)
  double p0 = 0.0;
  float s0 = 0.0f;
  bool fresh = false;       // incremental with a fresh front (reuse needs the same base)
};

void front(Chain& C) {
  const int64_t n = C.n;
  // tile totals (the look-back's values), in float like the kernel
  std::vector<float> tf(C.nk);
  for (int t = 0; t < C.nk; ++t) {
    double tot = 0.0;
    for (int64_t i = (int64_t)t * kTile; i < std::min<int64_t>(n, (int64_t)(t + 1) * kTile); ++i)
      if (!nf_flags(C.x.at(i))) tot += (double)C.x.at(i);
    tf.at(t) = getenv("EMU_ZERO_P") ? 0.0f : (float)tot;
  }
  for (int t = 0; t < C.nk; ++t) {
    const int64_t e0 = (int64_t)t * kTile;
    std::vector<float> xs(kTile + kW);
    for (int i = 0; i < kTile + kW; ++i) xs.at(i) = e0 + i < n ? C.x.at(e0 + i) : 0.0f;
    double P = C.p0;
    for (int i = 0; i < t; ++i)
      if (std::isfinite(tf.at(i))) P += (double)tf.at(i);
    std::vector<double> wsum(kBlocksPerTile);
    double ttotal = 0.0;
    for (int tid = 0; tid < kBlocksPerTile; ++tid) {
      const int b = t * kBlocksPerTile + tid;
      double s = 0.0;
      int fl = 0;
      for (int j = 0; j < kW; ++j) {
        const float e = xs.at(tid * kW + j);
        const int f = nf_flags(e);
        fl |= f;
        if (!f) s += (double)e;
      }
      if (b < C.nb) C.wflg.at(b) = (uint8_t)fl;
      wsum.at(tid) = s;
      ttotal += s;
    }
    std::vector<int> sbs(kBlocksPerTile + 1);
    std::vector<double> sA(kBlocksPerTile);
    double acc = 0.0;
    for (int tid = 0; tid < kBlocksPerTile; ++tid) {
      const int b = t * kBlocksPerTile + tid;
      const double wpre = P + acc;
      acc += wsum.at(tid);
      double best = wpre, run = wpre;
      int bj = -1;
      for (int j = 0; j < kW; ++j) {
        if (j >= kJLo && j <= kJHi && (bj < 0 || std::fabs(run) > std::fabs(best)) &&
            e0 + tid * kW + j < n) {
          best = run;
          bj = j;
        }
        const float e = xs.at(tid * kW + j);
        if (std::isfinite(e)) run += (double)e;
      }
      if (bj < 0) {
        best = wpre;
        bj = 0;
      }
      if (b == 0) {
        best = 0.0;
        bj = 0;
      }
      sbs.at(tid) = tid * kW + bj;
      sA.at(tid) = best;
    }
    {
      double r2 = P + ttotal, b2 = r2;
      int j2 = -1;
      for (int j = 0; j < kW; ++j) {
        if (j >= kJLo && j <= kJHi && (j2 < 0 || std::fabs(r2) > std::fabs(b2)) &&
            e0 + kTile + j < n) {
          b2 = r2;
          j2 = j;
        }
        const float e = xs.at(kTile + j);
        if (std::isfinite(e)) r2 += (double)e;
      }
      sbs.at(kBlocksPerTile) = kTile + (j2 < 0 ? 0 : j2);
    }
    for (int tid = 0; tid < kBlocksPerTile; ++tid) {
      const int b = t * kBlocksPerTile + tid;
      if (b < C.nb) C.bs.at(b) = (int)(e0 + sbs.at(tid));
      if (b == C.nb - 1) C.bs.at(C.nb) = (int)n;
    }
    // groups
    std::vector<double> gkey(kKW, -1.0);
    std::vector<int> gid(kKW, 0);
    for (int gi = 0; gi < kKW; ++gi) {
      double key = -1.0;
      int kid = INT32_MAX;
      for (int l = 0; l < kGW; ++l) {
        const int tid = gi * kGW + l;
        const int b = t * kBlocksPerTile + tid;
        const double k2 = b < C.nb ? (l >= kJLo && l <= kJHi ? std::fabs(sA.at(tid)) : -0.5) : -1.0;
        const int i2 = b < C.nb ? b : INT32_MAX;
        if (k2 > key || (k2 == key && i2 < kid)) {
          key = k2;
          kid = i2;
        }
      }
      const int q = t * kKW + gi;
      if (q < C.ng) {
        C.gs.at(q) = q == 0 ? 0 : kid;
        if (q == C.ng - 1) C.gs.at(C.ng) = C.nb;
      }
      gkey.at(gi) = q < C.ng ? key : -1.0;
      gid.at(gi) = q;
    }
    double bk = -2.0;
    int bq = 0;
    for (int i = 0; i < kKW; ++i) {
      const double k = i >= kJLo && i <= kJHi ? gkey.at(i) : (gkey.at(i) >= 0.0 ? -0.5 : -1.0);
      if (k > bk) {
        bk = k;
        bq = gid.at(i);
      }
    }
    C.ks.at(t) = t == 0 ? 0 : bq;
    if (t == C.nk - 1) C.ks.at(C.nk) = C.ng;
    double itot = 0.0;
    for (int tid = 0; tid < kBlocksPerTile; ++tid) {
      const int b = t * kBlocksPerTile + tid;
      if (b >= C.nb) continue;
      const int s0 = sbs.at(tid);
      const int s1 = b == C.nb - 1 ? (int)(n - e0) : sbs.at(tid + 1);
      const float G = b == 0 ? 0.0f : (float)sA.at(tid);
      float s = G;
      double fsum = 0.0;
      for (int i = s0; i < s1; ++i) {
        const float e = xs.at(i);
        s = s + e;
        if (std::isfinite(e)) fsum += (double)e;
      }
      const double incv = std::isfinite(s) && std::isfinite(G) ? (double)s - (double)G : fsum;
      C.inc.at(b) = incv;
      itot += incv;
    }
    C.tinc.at(t) = itot;
  }
}

// dirty: per block, 1 = its elements changed since the maps were built
// (nullptr: build everything).  Clean blocks keep their leaf maps, groups of
// clean blocks their group maps, superblocks of clean groups their maps --
// seqsum.hip's incremental rebuild (the guesses, boundaries and candidate
// bases stay those of the last full build).
void maps(Chain& C, const std::vector<uint8_t>* dirty = nullptr) {
  for (int k = 0; k < C.nk; ++k) {
    const int ga = C.ks.at(k), gb = C.ks.at(k + 1);
    const int ba = C.gs.at(ga), bb = C.gs.at(gb);
    bool sb_dirty = dirty == nullptr || C.fresh;
    if (dirty)
      for (int b = ba; b < bb; ++b) sb_dirty = sb_dirty || dirty->at(b);
    if (!sb_dirty) continue;
    const int ea = C.bs.at(ba), eb = C.bs.at(bb);
    const int ngr = gb - ga, nblk = bb - ba, nel = eb - ea;
    if (ngr < 1 || ngr > kMaxSbGroups || nblk < 1 || nblk > kMaxSbBlocks || nel < 1 || nel > kMaxSbElems)
      throw std::runtime_error("superblock size out of range");
    std::vector<float> xs(kMaxSbElems);
    for (int i = 0; i < nel; ++i) xs.at(i) = C.x.at(ea + i);
    std::vector<int> sbs(kMaxSbBlocks + 1), sgs(kMaxSbGroups + 1);
    for (int i = 0; i <= nblk; ++i) sbs.at(i) = C.bs.at(ba + i) - ea;
    for (int i = 0; i <= ngr; ++i) sgs.at(i) = C.gs.at(ga + i) - ba;
    const int tb = ba / kBlocksPerTile;
    double base = C.p0;
    for (int i = 0; i < tb; ++i) base += C.tinc.at(i);
    for (int b = tb * kBlocksPerTile; b < ba; ++b) base += C.inc.at(b);
    std::vector<double> Gd(kMaxSbBlocks + 1);
    double pre = 0.0;
    for (int i = 0; i < nblk; ++i) {
      Gd.at(i) = ba + i == 0 ? 0.0 : base + pre;
      pre += C.inc.at(ba + i);
    }
    std::vector<Leaf> lf(kMaxSbBlocks);
    std::vector<uint8_t> dirty_leaf(kMaxSbBlocks, 0);
    for (int bl = 0; bl < nblk; ++bl) {
      const float G = candidate_base((float)Gd.at(bl), kLeafR);
      if (dirty && !dirty->at(ba + bl) && (!C.fresh || std::memcmp(&G, &C.leaf.at(ba + bl).h.G, 4) == 0)) {
        lf.at(bl) = C.leaf.at(ba + bl);
        continue;
      }
      if (dirty) dirty_leaf.at(bl) = 1;
      C.work[0] += 1;
      const int e0 = grid_exp(G);
      // candidate 0 first: when its run rounds on no grid coarser than G's
      // (m = 0, ~99.7% of an ICP loop's blocks) it alone is the map; else
      // all kLeafR candidates as before
      Run p[kLeafR];
      run_init(p[0], cand(G, e0, 0));
      for (int i = sbs.at(bl); i < sbs.at(bl + 1); ++i) run_step(p[0], xs.at(i), e0);
      const bool more = p[0].need != kNoNeed && p[0].need > e0;
      for (int r = 1; r < kLeafR; ++r) {
        run_init(p[r], cand(G, e0, r));
        if (more)
          for (int i = sbs.at(bl); i < sbs.at(bl + 1); ++i) run_step(p[r], xs.at(i), e0);
      }
      int need = kNoNeed;
      for (int r = 0; r < (more ? kLeafR : 1); ++r) need = imax(need, p[r].need);
      const int mneed = need == kNoNeed ? 0 : imax(0, need - e0);
      const bool exact_only = mneed > kLeafM;
      const int m = exact_only ? 0 : mneed;
      if (getenv("EMU_MHIST")) {  // (statistics) leaf lattice: m 0..kLeafM, exact-only, opaque
        static long long h[8];
        static int calls;
        h[p[0].opaque ? 7 : (exact_only ? 6 : m)]++;
        if (++calls % 1000 == 0)
          std::fprintf(stderr, "mhist m0 %lld m1 %lld m2 %lld exact_only %lld opaque %lld\n", h[0], h[1], h[2], h[6], h[7]);
      }
      Leaf& o = lf.at(bl);
      o.h.G = G;
      o.h.e0 = e0;
      o.h.m = m;
      o.h.flags = p[0].opaque ? kOpaque : 0;
      for (int r = 0; r < kLeafR; ++r) {
        MapEnt en;
        en.E = p[r].s;
        en.LOu = lo_units((double)p[r].lo, e0);
        en.HIu = hi_units((double)p[r].hi, e0);
        if (p[r].opaque || r >= (1 << m)) {
          en.LOu = 1;
          en.HIu = 0;
        } else if (exact_only) {
          en.LOu = imax(en.LOu, 0);
          en.HIu = imin(en.HIu, 0);
        }
        o.e[r] = en;
      }
      C.leaf.at(ba + bl) = o;
    }
    std::vector<GroupMap> gm(kMaxSbGroups);
    bool any_group = false;
    for (int gi = 0; gi < ngr; ++gi) {
      const int c0 = sgs.at(gi), c1 = sgs.at(gi + 1);
      if (c1 - c0 < 1 || c1 - c0 > 2 * kGW - 1) throw std::runtime_error("group size out of range");
      bool g_dirty = dirty == nullptr;
      if (dirty)
        for (int j = c0; j < c1; ++j) g_dirty = g_dirty || dirty_leaf.at(j);
      if (!g_dirty) {
        gm.at(gi) = C.grp.at(ga + gi);
        continue;
      }
      C.work[1] += 1;
      any_group = true;
      const MapHdr h0 = lf.at(c0).h;
      int lat = h0.e0 + h0.m;
      for (int j = c0 + 1; j < c1; ++j) {
        const MapHdr hj = lf.at(j).h;
        if (!(hj.flags & kOpaque)) lat = imax(lat, hj.e0 + hj.m);
      }
      int m = imax(0, lat - h0.e0);
      const bool exact_only = m > kGroupM;
      if (getenv("EMU_MHIST")) {
        static long long h[8];
        static int calls;
        h[exact_only ? 7 : m]++;
        if (++calls % 10000 == 0)
          std::fprintf(stderr, "ghist %lld %lld %lld %lld %lld exact_only %lld\n", h[0], h[1], h[2], h[3], h[4], h[7]);
      }
      if (exact_only) m = 0;
      const int R = 1 << m;
      const float G = candidate_base(h0.G, R);
      const int e0 = grid_exp(G);
      GroupMap& o = gm.at(gi);
      o.h.G = G;
      o.h.e0 = e0;
      o.h.m = m;
      o.h.flags = 0;
      for (int r = 0; r < kGroupR; ++r) {
        MapEnt en;
        en.E = 0.0f;
        en.LOu = 1;
        en.HIu = 0;
        if (r < R) {
          float x = cand(G, e0, r);
          double clo = -INFINITY, chi = INFINITY;
          bool ok = true;
          for (int j = c0; j < c1 && ok; ++j) ok = through(x, clo, chi, lf.at(j).h, lf.at(j).e);
          if (ok) {
            if (exact_only) {
              clo = std::fmax(clo, 0.0);
              chi = std::fmin(chi, 0.0);
            }
            en.E = x;
            en.LOu = lo_units(clo, e0);
            en.HIu = hi_units(chi, e0);
          }
        }
        o.e[r] = en;
      }
      C.grp.at(ga + gi) = o;
    }
    if (dirty && !any_group) continue;
    C.work[2] += 1;
    {
      const MapHdr h0 = gm.at(0).h;
      int lat = h0.e0 + h0.m;
      for (int j = 1; j < ngr; ++j) lat = imax(lat, gm.at(j).h.e0 + gm.at(j).h.m);
      int m = imax(0, lat - h0.e0);
      const bool exact_only = m > kSbM;
      if (getenv("EMU_MHIST")) {
        static long long h[8];
        static int calls;
        h[exact_only ? 7 : m]++;
        if (++calls % 1000 == 0)
          std::fprintf(stderr, "sbhist %lld %lld %lld %lld %lld %lld %lld exact_only %lld\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
      }
      if (exact_only) m = 0;
      const int R = 1 << m;
      const float G = candidate_base(h0.G, R);
      const int e0 = grid_exp(G);
      SbMap& o = C.sbm.at(k);
      o.h.G = G;
      o.h.e0 = e0;
      o.h.m = m;
      o.h.flags = 0;
      for (int r = 0; r < kSbR; ++r) {
        MapEnt en;
        en.E = 0.0f;
        en.LOu = 1;
        en.HIu = 0;
        if (r < R) {
          float x = cand(G, e0, r);
          double clo = -INFINITY, chi = INFINITY;
          bool ok = true;
          for (int j = 0; j < ngr && ok; ++j) ok = through(x, clo, chi, gm.at(j).h, gm.at(j).e);
          if (ok) {
            if (exact_only) {
              clo = std::fmax(clo, 0.0);
              chi = std::fmin(chi, 0.0);
            }
            en.E = x;
            en.LOu = lo_units(clo, e0);
            en.HIu = hi_units(chi, e0);
          }
        }
        o.e[r] = en;
      }
    }
  }
}

bool walk_try(float& s, const MapHdr& h, const MapEnt* e, int nent) {
  if (h.flags & kOpaque) return false;
  int k;
  if (!offset_units(s, h, k)) return false;
  const int r = k & ((1 << h.m) - 1);
  if (r >= nent) throw std::runtime_error("residue out of range");
  float out;
  if (!apply_ent(k - r, h.e0, e[r], out)) return false;
  s = out;
  return true;
}

float walk(Chain& C) {
  float s = C.s0;
  int64_t pos_nf = -1;
  for (int k = 0; k < C.nk && pos_nf < 0; ++k) {
    ++C.stats[0];
    const float s_in = s;
    if (walk_try(s, C.sbm.at(k).h, C.sbm.at(k).e, kSbR)) {
      ++C.stats[1];
      continue;
    }
    if (getenv("EMU_MISS")) {  // (statistics) why superblock k's map missed
      const MapHdr& h = C.sbm.at(k).h;
      const double du = ((double)s_in - (double)h.G) / std::ldexp(1.0, h.e0);
      int kk = 0;
      const bool off = offset_units(s_in, h, kk);
      const int r = off ? (kk & ((1 << h.m) - 1)) : -1;
      std::fprintf(stderr, "miss k=%d s=%.9g G=%.9g e0=%d m=%d fl=%d units=%.1f off=%d r=%d win=[%d,%d] du=%d\n", k,
                   (double)s_in, (double)h.G, h.e0, h.m, h.flags, du, (int)off, r,
                   r >= 0 ? C.sbm.at(k).e[r].LOu : 0, r >= 0 ? C.sbm.at(k).e[r].HIu : 0, off ? kk - r : 0);
    }
    const int ga = C.ks.at(k), gb = C.ks.at(k + 1);
    for (int q = ga; q < gb && pos_nf < 0; ++q) {
      ++C.stats[2];
      if (walk_try(s, C.grp.at(q).h, C.grp.at(q).e, kGroupR)) {
        ++C.stats[3];
        continue;
      }
      for (int b = C.gs.at(q); b < C.gs.at(q + 1); ++b) {
        ++C.stats[4];
        if (walk_try(s, C.leaf.at(b).h, C.leaf.at(b).e, kLeafR)) {
          ++C.stats[5];
          continue;
        }
        ++C.stats[6];
        const int e0 = C.bs.at(b), e1 = C.bs.at(b + 1);
        if (e1 - e0 > 2 * kW) throw std::runtime_error("block size out of range");
        for (int i = e0; i < e1; ++i) s = s + C.x.at(i);
        if (!std::isfinite(s)) {
          pos_nf = e1;
          break;
        }
      }
    }
  }
  if (pos_nf >= 0) {
    int64_t i = pos_nf;
    for (; i < C.n && (i % kW) != 0; ++i) s = s + C.x.at(i);
    int orf = 0;
    for (int64_t w = i / kW; w < C.nb; ++w) orf |= C.wflg.at(w);
    if (std::isnan(s) || (orf & 1) || (s > 0 && (orf & 4)) || (s < 0 && (orf & 2))) s = NAN;
  }
  return s;
}

}  // namespace

// seqsum_emu <in.f32> <n> <nch> [nstreams [incremental]]: nstreams float4
// streams of n rows back to back (an ICP loop's iterations); incremental: a
// stream after the first rebuilds only the maps of blocks whose windows
// changed (the GPU's rule: block b is dirty when window b or b + 1 is).
// One line per stream and chain: sum bits, walk stats, maps built.
int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: seqsum_emu <in.f32> <n> <nch> [nstreams [incremental]]\n");
    return 2;
  }
  const int64_t n = std::atoll(argv[2]);
  const int nch = std::atoi(argv[3]);
  const int ns = argc > 4 ? std::atoi(argv[4]) : 1;
  const int incr_mode = argc > 5 ? std::atoi(argv[5]) : 0;  // 1 stale front, 2 fresh front
  const bool incr = incr_mode != 0;
  std::vector<float> raw((size_t)n * 4 * ns);
  FILE* f = std::fopen(argv[1], "rb");
  if (!f || std::fread(raw.data(), 4, raw.size(), f) != raw.size()) {
    std::fprintf(stderr, "read failed\n");
    return 2;
  }
  std::fclose(f);
  try {
    std::vector<Chain> chains(nch);
    for (int si = 0; si < ns; ++si) {
      for (int c = 0; c < nch; ++c) {
        Chain& C = chains[c];
        const bool inc_now = incr && si > 0 && n > 0;
        std::vector<uint8_t> dirty;
        if (inc_now) {
          std::vector<uint8_t> dw(C.nb + 1, 0);
          for (int64_t i = 0; i < n; ++i) {
            const float v = raw[((size_t)si * n + i) * 4 + c];
            uint32_t a, b;
            std::memcpy(&a, &v, 4);
            std::memcpy(&b, &C.x.at(i), 4);
            if (a != b) dw.at(i / kW) = 1;
            C.x.at(i) = v;
          }
          dirty.assign(C.nb, 0);
          for (int b = 0; b < C.nb; ++b) dirty.at(b) = dw.at(b) | dw.at(b + 1);
          for (int w = 0; w < C.nb; ++w) {  // the window flags stay current
            int fl = 0;
            for (int64_t i = (int64_t)w * kW; i < std::min<int64_t>(n, (int64_t)(w + 1) * kW); ++i)
              fl |= nf_flags(C.x.at(i));
            C.wflg.at(w) = (uint8_t)fl;
          }
        } else {
          C = Chain();
          C.n = n;
          C.nb = (int)((n + kW - 1) / kW);
          C.ng = (C.nb + kGW - 1) / kGW;
          C.nk = (C.ng + kKW - 1) / kKW;
          C.x.resize(n);
          for (int64_t i = 0; i < n; ++i) C.x[i] = raw[((size_t)si * n + i) * 4 + c];
          C.wflg.assign(C.nb, 0);
          C.inc.assign(C.nb, 0.0);
          C.tinc.assign(C.nk, 0.0);
          C.bs.assign(C.nb + 1, -1);
          C.gs.assign(C.ng + 1, -1);
          C.ks.assign(C.nk + 1, -1);
          C.leaf.resize(C.nb);
          C.grp.resize(C.ng);
          C.sbm.resize(C.nk);
        }
        for (int j = 0; j < 8; ++j) C.stats[j] = 0;
        for (int j = 0; j < 3; ++j) C.work[j] = 0;
        // EMU_P0="p,p,p,p" (fp64) / EMU_S0="hex,hex,hex,hex" (float bits): a stretch
        // of a longer chain, per chain
        if (const char* e = getenv("EMU_P0")) {
          const char* q = e;
          for (int j = 0; j < c && q; ++j) q = std::strchr(q, ',') ? std::strchr(q, ',') + 1 : nullptr;
          C.p0 = q ? std::strtod(q, nullptr) : 0.0;
        }
        if (const char* e = getenv("EMU_S0")) {
          const char* q = e;
          for (int j = 0; j < c && q; ++j) q = std::strchr(q, ',') ? std::strchr(q, ',') + 1 : nullptr;
          const uint32_t u = q ? (uint32_t)std::strtoul(q, nullptr, 16) : 0u;
          std::memcpy(&C.s0, &u, 4);
        }
        float s = C.s0;
        if (n > 0) {
          C.fresh = inc_now && incr_mode == 2;
          if (!inc_now || C.fresh) {
            front(C);
            if (const char* dump = getenv("EMU_DUMP")) {
              // the front kernel's tables of chain c: bs, gs, ks (int32), inc (f64)
              char path[512];
              std::snprintf(path, sizeof(path), "%s.%d", dump, c);
              FILE* g = std::fopen(path, "wb");
              std::fwrite(C.bs.data(), 4, C.bs.size(), g);
              std::fwrite(C.gs.data(), 4, C.gs.size(), g);
              std::fwrite(C.ks.data(), 4, C.ks.size(), g);
              std::fwrite(C.inc.data(), 8, C.inc.size(), g);
              std::fclose(g);
            }
          }
          maps(C, inc_now ? &dirty : nullptr);
          s = walk(C);
        }
        uint32_t u;
        std::memcpy(&u, &s, 4);
        std::printf("%08x %d %d %d %d %d %d %d %d %d %d\n", u, C.stats[0], C.stats[1], C.stats[2],
                    C.stats[3], C.stats[4], C.stats[5], C.stats[6], C.work[0], C.work[1], C.work[2]);
      }
    }
  } catch (const std::exception& e) {
    std::printf("ERROR %s\n", e.what());
    return 1;
  }
  return 0;
}
