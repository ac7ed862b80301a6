"""Per-iteration durations of the ICP kernels from a rocprofv3 kernel trace
of a single-pair-in-flight bench (scripts: prof of bench.py --inflight 1).
  python scripts/iter_profile.py TRACE.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
it, per, pairs = -1, {}, 0
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    if "k_init_state" in n:
        it = 0
        pairs += 1
        continue
    if it < 0 or "P2Point" not in n:
        continue
    k = 0 if "k_icp_nn<" in n else (1 if "k_icp_fb<" in n else (
        2 if "k_icp_pix<" in n else (3 if "k_reduce_solve<" in n else -1)))
    if k < 0:
        continue
    per.setdefault(it, [0.0, 0.0, 0.0, 0.0])[k] += d
    if k == 3:
        it += 1
print(f"pairs {pairs}; per-pair us: iter nn fb pix solve")
for i in list(range(0, 8)) + [16, 32, 64, 127]:
    if i in per:
        print(i, " ".join(f"{x / pairs:8.1f}" for x in per[i]))
tot = sum(sum(v) for v in per.values())
print("per pair total us", round(tot / pairs), "first 4 iterations share",
      round(sum(sum(per[i]) for i in range(4) if i in per) / tot, 3))
