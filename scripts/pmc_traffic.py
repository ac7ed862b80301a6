"""HBM traffic per ICP iteration of the NN pass -- k_icp_nn<Acc> and
k_icp_fb<Acc> (Acc = RefAcc, the bench value's mode, or P2PointAcc: the
optional 4th argument), per launch each and summed -- from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; counter_collection.csv each), corrected as
/opt/skills/guides/MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE (KiB) x 2
on gfx950, WRITE_SIZE (KiB) as is.  Writes the JSON bench.py reads, stamped
with the library's source hash (lib/BUILD_INFO.json): bench.py reports the
traffic only while it matches the library it runs.

A batched run (k_icp_nn_b / k_icp_fb_b: one launch per batch of PAIRS frame
pairs, every batch full) is divided by PAIRS: the JSON holds bytes per pair
iteration, bench.py scales them by its pairs per launch.

CONFIG (optional 6th argument, bench.py's workload key, e.g.
stream_1280x720_p2point_ref or stream_640x480_p2plane; default the value's
stream_640x480_p2point_ref) stamps the workload the pass measured.

  python scripts/pmc_traffic.py OUT.json FETCH.csv WRITE.csv [RefAcc|P2PointAcc|P2PlaneAcc] [PAIRS] [CONFIG]"""
import csv
import json
import sys

ACC = sys.argv[4] if len(sys.argv) > 4 else "RefAcc"
PAIRS = int(sys.argv[5]) if len(sys.argv) > 5 else 1
CONFIG = sys.argv[6] if len(sys.argv) > 6 else "stream_640x480_p2point_ref"


def per_dispatch(path, counter, kernel):
    vals = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if r["Counter_Name"] != counter or kernel not in name or ACC not in name:
            continue
        # one row per (dispatch, counter); sum any per-dimension rows
        key = r.get("Dispatch_Id") or r.get("Correlation_Id") or len(vals)
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    v = sorted(vals.values())
    return v


def main():
    out, fpath, wpath = sys.argv[1:4]
    d = {"kernels": {}, "note": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as is; rocprofv3 --pmc, "
                                "separate passes; per launch, " + ACC + " instances"}
    tot = 0.0
    batched = any("k_icp_nn_b<" in r["Kernel_Name"] for r in csv.DictReader(open(fpath)))
    kernels = ("k_icp_nn_b<", "k_icp_fb_b<") if batched else ("k_icp_nn<", "k_icp_fb<")
    d["pairs_per_launch"] = PAIRS if batched else 1
    for k in kernels:
        f = per_dispatch(fpath, "FETCH_SIZE", k)
        w = per_dispatch(wpath, "WRITE_SIZE", k)
        if not f or not w:
            raise SystemExit(f"no {k}{ACC}> rows")
        fm = sum(f) / len(f) * 1024.0 * 2.0  # KiB -> B, gfx950 half-count correction
        wm = sum(w) / len(w) * 1024.0
        d["kernels"][k.rstrip("<")] = {"dispatches": [len(f), len(w)],
                                       "fetch_bytes_corrected": fm, "write_bytes": wm,
                                       "bytes_per_launch": fm + wm,
                                       "fetch_size_kib_median_raw": f[len(f) // 2]}
        tot += fm + wm
    d["config"] = CONFIG
    d["nn_pass_bytes_per_iteration"] = tot  # per launch
    d["nn_pass_bytes_per_pair_iteration"] = tot / d["pairs_per_launch"]
    try:
        d["source_hash"] = json.load(open("realsensetracker_amd/lib/BUILD_INFO.json"))["source_hash"]
    except (OSError, KeyError, ValueError):
        d["source_hash"] = None
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
