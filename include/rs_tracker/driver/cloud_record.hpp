// rs_tracker/driver/cloud_record.hpp -- on-disk frame records for the replay
// path.  The reference records one protobuf
// cho::proto::core::geometry::PointCloud per frame (rs_viewer.cpp:104-112)
// and replays a glob of them (rs_replay_app.cpp:211-225); that schema lives
// in the unvendored cho_util, so the build defines a raw record instead:
//
//   offset  0  char[4]  "RSTC"
//           4  uint32   version (1)
//           8  uint64   n, points
//          16  float64  stamp (seconds)
//          24  uint32   flags (0)
//          28  uint32   reserved (0)
//          32  float32  xyz[n][3]   (Cloud3f's bytes: 3 x n column-major)
//
// little-endian, one frame per file; realsensetracker_amd/records.py reads
// and writes the same bytes.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "rs_tracker/common/types.hpp"

namespace rs_tracker {

struct CloudRecordHeader {
  char magic[4];
  uint32_t version;
  uint64_t n;
  double stamp;
  uint32_t flags;
  uint32_t reserved;
};
static_assert(sizeof(CloudRecordHeader) == 32, "record header is 32 bytes");

inline bool WriteCloudRecord(const std::string& path, const Cloud3f& cloud, double stamp = 0.0) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  CloudRecordHeader h{{'R', 'S', 'T', 'C'}, 1u, (uint64_t)cloud.cols(), stamp, 0u, 0u};
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  const size_t nf = 3 * (size_t)cloud.cols();
  if (ok && nf) ok = std::fwrite(cloud.data(), sizeof(float), nf, f) == nf;
  return std::fclose(f) == 0 && ok;
}

inline bool ReadCloudRecord(const std::string& path, Cloud3f* cloud, double* stamp = nullptr) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  CloudRecordHeader h{};
  bool ok = std::fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, "RSTC", 4) == 0 &&
            h.version == 1u && h.n < ((uint64_t)1 << 34);
  if (ok) {
    Cloud3f c((int64_t)h.n);
    const size_t nf = 3 * (size_t)h.n;
    ok = nf == 0 || std::fread(c.data(), sizeof(float), nf, f) == nf;
    if (ok) {
      *cloud = std::move(c);
      if (stamp) *stamp = h.stamp;
    }
  }
  std::fclose(f);
  return ok;
}

}  // namespace rs_tracker
