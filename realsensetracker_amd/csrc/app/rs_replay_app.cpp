// rs_replay_app -- the reference's frame-to-frame replay loop
// (rs_tracker/app/src/rs_replay_app.cpp:211-270) as host C++ over the
// MI355X align module.  Frames come from a directory of recorded RSTC
// records (include/rs_tracker/driver/cloud_record.hpp; the reference replays
// a glob of protobuf records) or from the synthetic scene (driver decoupled
// from the camera):
//
//   for each frame: cloud_raw (record, or depth -> rst_unproject)
//     RemoveNans(cloud_raw, &cloud)                                 (:229)
//     first frame: prev = cloud; acc.AddCloud(total_xfm, prev)       (:237-241)
//     DownsampleVoxel(cloud, v, &curr_down), (prev, v, &prev_down)  (:246-247)
//     xfm = Identity; ok = AlignIcp3d(curr_down, prev_down, 128, &xfm) (:235,251)
//     if ok: total_xfm = total_xfm * xfm; acc.AddCloud(total_xfm, cloud);
//            prev = cloud                                            (:264-269)
//
// Prints per-frame timing and, for the synthetic scene, drift against the
// ground truth.
//
//   rs_replay_app [--frames N] [--width W] [--height H] [--iters K] [--seed S]
//                 [--voxel-mm V]  (voxel edge in mm, default 50 as the
//                                  reference; 0 = align the full clouds)
//                 [--dump FILE]   (per-frame xfm, one line of 16 col-major floats)
//                 [--records DIR] (replay DIR/*.rstc in name order)
//                 [--write-records DIR] (record the synthetic stream's raw clouds)
//                 [--accum-mm V --map-out FILE] (CloudAccumulator voxel, written
//                                  as one record at the end)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <memory>
#include <string>
#include <vector>

#include "rs_tracker/align/align_icp.hpp"
#include "rs_tracker/common/cloud_accumulator.hpp"
#include "rs_tracker/common/point_cloud_utils.hpp"
#include "rs_tracker/driver/cloud_record.hpp"

namespace {

struct Args {
  int frames = 10, width = 640, height = 480, iters = 128, voxel_mm = 50;
  uint64_t seed = 0;
  const char* dump = nullptr;  // write each frame's xfm (16 floats, col-major)
  const char* records = nullptr;
  const char* write_records = nullptr;
  int accum_mm = 0;
  const char* map_out = nullptr;
};

Args Parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i];
    const long v = std::strtol(argv[i + 1], nullptr, 10);
    if (k == "--frames") a.frames = (int)v;
    else if (k == "--width") a.width = (int)v;
    else if (k == "--height") a.height = (int)v;
    else if (k == "--iters") a.iters = (int)v;
    else if (k == "--seed") a.seed = (uint64_t)v;
    else if (k == "--dump") a.dump = argv[i + 1];
    else if (k == "--voxel-mm") a.voxel_mm = (int)v;
    else if (k == "--records") a.records = argv[i + 1];
    else if (k == "--write-records") a.write_records = argv[i + 1];
    else if (k == "--accum-mm") a.accum_mm = (int)v;
    else if (k == "--map-out") a.map_out = argv[i + 1];
    else { std::fprintf(stderr, "unknown flag %s\n", k.c_str()); std::exit(2); }
  }
  return a;
}

// inverse of a rigid 4x4 column-major transform
void RigidInverse(const float* T, float* out) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) out[c * 4 + r] = T[r * 4 + c];
  for (int r = 0; r < 3; ++r) {
    float s = 0.f;
    for (int k = 0; k < 3; ++k) s += out[k * 4 + r] * T[12 + k];
    out[12 + r] = -s;
  }
  out[3] = out[7] = out[11] = 0.f;
  out[15] = 1.f;
}

void Mul(const float* A, const float* B, float* out) {
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      float s = 0.f;
      for (int k = 0; k < 4; ++k) s += A[k * 4 + r] * B[c * 4 + k];
      out[c * 4 + r] = s;
    }
}

void PoseError(const float* T, const float* G, double* ang, double* tr) {
  double tr3 = 0.0;  // trace(R_T R_G^T)
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) tr3 += (double)T[c * 4 + r] * G[c * 4 + r];
  *ang = std::acos(std::fmax(-1.0, std::fmin(1.0, (tr3 - 1.0) / 2.0)));
  double s = 0.0;
  for (int r = 0; r < 3; ++r) s += (double)(T[12 + r] - G[12 + r]) * (T[12 + r] - G[12 + r]);
  *tr = std::sqrt(s);
}

}  // namespace

int main(int argc, char** argv) {
  using rs_tracker::gpu::Check;
  Args a = Parse(argc, argv);
  std::vector<std::string> files;
  if (a.records) {
    for (const auto& e : std::filesystem::directory_iterator(a.records))
      if (e.path().extension() == ".rstc") files.push_back(e.path().string());
    std::sort(files.begin(), files.end());
    a.frames = (int)files.size();
    if (a.frames < 1) {
      std::fprintf(stderr, "no .rstc records in %s\n", a.records);
      return 2;
    }
  }
  if (a.write_records) std::filesystem::create_directories(a.write_records);
  rst_scene* scene = nullptr;
  Check(rst_scene_create(a.seed, &scene), "rst_scene_create");
  rst_intrinsics K{};
  K.width = a.width;
  K.height = a.height;
  K.fx = K.fy = 385.0f * (float)a.width / 640.0f;
  K.cx = 0.5f * (float)a.width;
  K.cy = 0.5f * (float)a.height;
  K.depth_scale = 0.001f;
  K.min_depth = 0.3f;
  K.max_depth = 5.0f;
  rs_tracker::gpu::Context& ctx = rs_tracker::gpu::DefaultContext();

  std::vector<uint16_t> depth((size_t)a.width * a.height);
  std::vector<float> xyz(3 * depth.size());
  auto grab = [&](int f, float* T_wc) {
    if (!files.empty()) {  // a recorded frame (:221-225)
      rs_tracker::Cloud3f cloud_raw, cloud;
      if (!rs_tracker::ReadCloudRecord(files[f], &cloud_raw)) {
        std::fprintf(stderr, "bad record %s\n", files[f].c_str());
        std::exit(2);
      }
      for (int k = 0; k < 16; ++k) T_wc[k] = (k % 5 == 0) ? 1.f : 0.f;
      rs_tracker::RemoveNans(cloud_raw, &cloud);  // (:229)
      return cloud;
    }
    Check(rst_scene_trajectory(scene, f, T_wc), "trajectory");
    Check(rst_scene_render_depth(scene, T_wc, &K, 1000u + (uint64_t)f, 0.001f, 0.03f, depth.data()),
          "render");
    int64_t n = 0;
    Check(rst_unproject(ctx.get(), depth.data(), &K, 0, xyz.data(), &n), "rst_unproject");
    const rs_tracker::Cloud3f cloud_raw(xyz.data(), n);
    if (a.write_records) {
      char name[64];
      std::snprintf(name, sizeof(name), "/frame_%05d.rstc", f);
      if (!rs_tracker::WriteCloudRecord(std::string(a.write_records) + name, cloud_raw, f / 30.0))
        std::exit(3);
    }
    rs_tracker::Cloud3f cloud;
    rs_tracker::RemoveNans(cloud_raw, &cloud);  // (:229)
    return cloud;
  };
  const float voxel = (float)a.voxel_mm / 1000.0f;  // 50 -> 0.05f exactly as the reference

  float T0[16], T0inv[16], Tf[16];
  rs_tracker::Cloud3f prev = grab(0, T0);
  RigidInverse(T0, T0inv);
  rs_tracker::Isometry3f total_xfm = rs_tracker::Isometry3f::Identity();
  std::unique_ptr<rs_tracker::CloudAccumulator> acc;
  if (a.accum_mm > 0) {
    acc.reset(new rs_tracker::CloudAccumulator((float)a.accum_mm / 1000.0f));
    acc->AddCloud(total_xfm, prev);  // (:240)
  }
  double worst_ang = 0.0, worst_tr = 0.0, total_ms = 0.0;
  int ok_count = 0;
  FILE* dump = a.dump ? std::fopen(a.dump, "w") : nullptr;
  for (int f = 1; f < a.frames; ++f) {
    rs_tracker::Cloud3f cloud = grab(f, Tf);
    rs_tracker::Isometry3f xfm = rs_tracker::Isometry3f::Identity();
    const auto t0 = std::chrono::steady_clock::now();
    bool suc;
    if (voxel > 0.f) {  // (:245-251)
      rs_tracker::Cloud3f curr_cloud_down, prev_cloud_down;
      rs_tracker::DownsampleVoxel(cloud, voxel, &curr_cloud_down);
      rs_tracker::DownsampleVoxel(prev, voxel, &prev_cloud_down);
      suc = rs_tracker::AlignIcp3d(curr_cloud_down, prev_cloud_down, a.iters, &xfm);
    } else {
      suc = rs_tracker::AlignIcp3d(cloud, prev, a.iters, &xfm);
    }
    const double ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    total_ms += ms;
    if (dump) {
      float x[16];
      rs_tracker::ToColMajor(xfm, x);
      for (int k = 0; k < 16; ++k) std::fprintf(dump, "%.9g%c", x[k], k == 15 ? '\n' : ' ');
    }
    if (suc) {
      total_xfm = total_xfm * xfm;
      if (acc) acc->AddCloud(total_xfm, cloud);  // (:266)
      prev = std::move(cloud);
      ++ok_count;
    } else {
      std::printf("ALIGNMENT FAILED!!\n");
    }
    float tot[16], gt[16];
    rs_tracker::ToColMajor(total_xfm, tot);
    Mul(T0inv, Tf, gt);
    double ang = 0.0, tr = 0.0;
    if (files.empty()) {  // ground truth only for the synthetic scene
      PoseError(tot, gt, &ang, &tr);
      worst_ang = std::fmax(worst_ang, ang);
      worst_tr = std::fmax(worst_tr, tr);
    }
    std::printf("frame %3d  n=%7lld  align %8.2f ms  drift %.2e rad %.2e m\n", f,
                (long long)prev.cols(), ms, ang, tr);
  }
  std::printf("frames %d  aligned %d  mean align %.2f ms  worst drift %.2e rad %.2e m\n",
              a.frames - 1, ok_count, total_ms / std::max(1, a.frames - 1), worst_ang, worst_tr);
  if (dump) std::fclose(dump);
  if (acc) {
    const rs_tracker::Cloud3f map = acc->ExtractPointCloud();
    std::printf("map points %lld\n", (long long)map.cols());
    if (a.map_out && !rs_tracker::WriteCloudRecord(a.map_out, map)) return 3;
  }
  rst_scene_destroy(scene);
  return ok_count == a.frames - 1 ? 0 : 1;
}
