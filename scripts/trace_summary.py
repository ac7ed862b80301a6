"""Summarise a rocprofv3 kernel_trace.csv: per-kernel average duration and
the gaps between consecutive kernels of the ICP loop.

    python scripts/trace_summary.py gpurun_out/prof_x/run_kernel_trace.csv
"""
import collections
import csv
import re
import statistics
import sys


def short(n):
    n = n.replace("rst::(anonymous namespace)::", "").replace("rst::", "")
    return re.sub(r"\(.*", "", n)[:48]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = collections.defaultdict(list)
for r in rows:
    dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':48s} {'calls':>6s} {'avg_us':>8s} {'med_us':>8s} {'min':>7s} {'max':>8s} {'tot_ms':>8s}")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:16]:
    print(f"{k:48s} {len(v):6d} {statistics.mean(v):8.2f} {statistics.median(v):8.2f} "
          f"{min(v):7.2f} {max(v):8.2f} {sum(v)/1e3:8.2f}")
gaps = collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    gaps[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append(
        (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
print("\ngaps (end -> next start), us")
for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:8]:
    print(f"  {k[0][:30]:30s} -> {k[1][:30]:30s} n={len(v):5d} med={statistics.median(v):7.2f}")
# ICP iteration period: start of k_icp_nn to the next
st = [int(r["Start_Timestamp"]) for r in rows if "k_icp_nn" in r["Kernel_Name"]]
per = [(b - a) / 1e3 for a, b in zip(st, st[1:]) if (b - a) < 5e6]
if per:
    print(f"\nICP iteration period: median {statistics.median(per):.1f} us, mean {statistics.mean(per):.1f} us over {len(per)}")
