"""HBM traffic per launch of k_icp_nn<P2PointAcc> from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; counter_collection.csv each), corrected as
/opt/skills/guides/MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE (KiB) x 2
on gfx950, WRITE_SIZE (KiB) as is.  Writes the JSON bench.py reads.

  python scripts/pmc_traffic.py OUT.json FETCH.csv WRITE.csv"""
import csv
import json
import sys

KERNEL = "k_icp_nn<rst::(anonymous namespace)::P2PointAcc>"


def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if r["Counter_Name"] != counter or "k_icp_nn<" not in name or "P2PointAcc" not in name:
            continue
        # one row per (dispatch, counter); sum any per-dimension rows
        key = r.get("Dispatch_Id") or r.get("Correlation_Id") or len(vals)
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    v = sorted(vals.values())
    return v


def main():
    out, fpath, wpath = sys.argv[1:4]
    f = per_dispatch(fpath, "FETCH_SIZE")
    w = per_dispatch(wpath, "WRITE_SIZE")
    if not f or not w:
        raise SystemExit("no k_icp_nn<P2PointAcc> rows")
    fm = sum(f) / len(f) * 1024.0 * 2.0  # KiB -> B, gfx950 half-count correction
    wm = sum(w) / len(w) * 1024.0
    d = {"kernel": KERNEL, "dispatches": [len(f), len(w)],
         "fetch_bytes_per_launch_corrected": fm, "write_bytes_per_launch": wm,
         "k_icp_nn_bytes_per_launch": fm + wm,
         "fetch_size_kib_median_raw": f[len(f) // 2],
         "note": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as is; rocprofv3 --pmc, separate passes"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
