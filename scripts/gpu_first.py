"""First end-to-end GPU check: NN bit-exactness, ICP parity, timing."""
import sys, time, numpy as np
sys.path.insert(0, '.')
from realsensetracker_amd import driver, align as A, _lib as L
from oracle import oracle as O

def err(T, D):
    dR = T[:3,:3].astype(np.float64) @ D[:3,:3].T
    return float(np.arccos(np.clip((np.trace(dR)-1)/2, -1, 1))), float(np.linalg.norm(T[:3,3]-D[:3,3]))

print("devices", L.device_count(), flush=True)
ctx = A.get_context(0)
for W, H in [(160, 120), (320, 240)]:
    K = driver.intrinsics(W, H)
    sc = driver.SyntheticScene(0)
    da, db, D = driver.make_pair(sc, K, seed=1)
    K4 = [K.fx, K.fy, K.cx, K.cy]
    pa = O.unproject(da, K4); pb = O.unproject(db, K4)
    pa_g = driver.unproject(da, K)
    print(W, H, "unproject bitexact", pa.shape == pa_g.shape and np.array_equal(pa, pa_g), flush=True)
    t0 = time.time(); tgt = A.Target.build(pa); print("build s", time.time()-t0, flush=True)
    # NN at identity and at GT
    for T in [np.eye(4, dtype=np.float32), D.astype(np.float32)]:
        q = O.transform_points(T, pb)
        gi, gd = tgt.query(q)
        oi, od = O.nn_bruteforce(pa, q)
        print(" nn idx eq", np.mean(gi == oi), "d2 eq", np.mean(gd == od), flush=True)
    # ICP p2point
    ok_o, T_o, mc_o, _ = O.align_icp(pb, pa, 128)
    T_g = np.eye(4, dtype=np.float32)
    t0 = time.time(); ok_g = A.AlignIcp3d(pb, pa, tgt, 128, T_g); tg = time.time() - t0
    print(" icp ok", ok_o, ok_g, "gpu-vs-oracle", err(T_g, T_o.astype(np.float64)), "gpu-vs-gt", err(T_g, D), "oracle-vs-gt", err(T_o, D), "gpu s", tg, flush=True)
    # normals + p2plane
    tgt.compute_normals(16)
    ng = tgt.normals()
    no = O.compute_normals(pa, 16)
    cosang = np.sum(ng * no, 1)
    print(" normals cos>0.9999", np.mean(cosang > 0.9999), "min", cosang.min(), flush=True)
    it_o, T2o, mc2 = O.align_p2plane(pb, pa, no, 30, 1e-6, 4e-4, 0.0)
    opts = L.default_opts(mode=L.RST_P2PLANE, max_iter=30)
    srct = A.Target.build(pb)
    r = A.align_prepared(srct, tgt, None, opts)
    print(" p2plane it", it_o, r.iterations, "gpu-vs-oracle", err(r.pose, T2o.astype(np.float64)), "gpu-vs-gt", err(r.pose, D), flush=True)
