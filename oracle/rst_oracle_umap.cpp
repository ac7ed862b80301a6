// rst_oracle_umap.cpp -- TEST INFRASTRUCTURE ONLY (see rst_oracle.h): the
// iteration order of the reference's std::unordered_map voxel tables, from a
// real std::unordered_map of this toolchain's libstdc++ (GCC 11).
//
// DownsampleVoxel (point_cloud_utils.cpp:34-68) emits its points by
// iterating `std::unordered_map<Eigen::Vector3i, int, MatrixHash>` (:54-57,
// :63-66); CloudAccumulator::ExtractPointCloud (rs_replay_app.cpp:112-121)
// iterates `std::unordered_map<Eigen::Array3i, Eigen::Vector3f, VoxelHash>`.
// Both tables only ever receive new keys (find, then emplace), in input
// order.  Both hashes are boost::hash_combine over the key's three ints:
//   MatrixHash (point_cloud_utils.cpp:13-22): hash_combine(seed, std::hash<int>()(k_i))
//   VoxelHash  (rs_replay_app.cpp:78-84):     hash_combine(seed, k_i)
// with std::hash<int> = static_cast<size_t> (libstdc++) and Boost's
// hash_value(int) = static_cast<size_t> as well, so both are
//   seed = 0; seed ^= size_t(k_i) + 0x9e3779b9 + (seed << 6) + (seed >> 2)
// -- the classic hash_combine of Boost <= 1.80 (Ubuntu 18.04 / 20.04 ship
// 1.65 / 1.71; 1.81 replaced the mixing step).  That version is the one
// unpinned assumption; the container itself is the real one.
#include <cstddef>
#include <cstdint>
#include <unordered_map>

namespace {

struct Key {
  int32_t x, y, z;
  bool operator==(const Key& o) const { return x == o.x && y == o.y && z == o.z; }
};

struct ClassicHash {
  std::size_t operator()(const Key& k) const noexcept {
    std::size_t seed = 0;
    const int32_t v[3] = {k.x, k.y, k.z};
    for (int i = 0; i < 3; ++i) seed ^= static_cast<std::size_t>(v[i]) + 0x9e3779b9 + (seed << 6) + (seed >> 2);
    return seed;
  }
};

}  // namespace

extern "C" {

// keys: n distinct int triples in insertion order.  order[k] = the insertion
// index of the k-th element a std::unordered_map iteration visits.
void orc_umap_order(const int32_t* keys, int64_t n, int64_t* order) {
  std::unordered_map<Key, int64_t, ClassicHash> m;
  for (int64_t i = 0; i < n; ++i) {
    const Key k{keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]};
    if (m.find(k) == m.end()) m.emplace(k, i);
  }
  int64_t j = 0;
  for (const auto& kv : m) order[j++] = kv.second;
}

// the container's bucket counts as n distinct keys arrive one by one:
// (elements before the insert that rehashed, new bucket count) pairs,
// returns the number of pairs (at most cap written)
int64_t orc_umap_schedule(int64_t n, int64_t* out, int64_t cap) {
  std::unordered_map<int64_t, int> m;  // (bucket policy: independent of key and hash)
  std::size_t nb = m.bucket_count();
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i) {
    m.emplace(i, 0);
    if (m.bucket_count() != nb) {
      nb = m.bucket_count();
      if (k < cap) {
        out[2 * k] = i;
        out[2 * k + 1] = (int64_t)nb;
      }
      ++k;
    }
  }
  return k;
}

}  // extern "C"
