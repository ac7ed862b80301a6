"""kNN-16 normals (ComputeNormals, point_cloud_utils.cpp:176-216) of 640x480
frame targets: run under rocprofv3 --kernel-trace --stats for k_normals_grid
(pixel windows) against k_normals (the BVH search, RST_KNN_GRID=0).
  python tools/normals_prof.py [frames]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from realsensetracker_amd import align as A  # noqa: E402
from realsensetracker_amd import driver  # noqa: E402

ctx = A.get_context(0)
K = driver.intrinsics(640, 480)
sc = driver.SyntheticScene(0)
nf = int(sys.argv[1]) if len(sys.argv) > 1 else 8
for i in range(nf):
    d = A.DeviceBuffer.from_array(sc.render(sc.trajectory(i), K, noise_seed=i), ctx)
    t = A.Target.from_depth_device(d.ptr, K, 16, ctx)
    ctx.synchronize()
    t.free()
    d.free()
print("ok", nf, "frames")
