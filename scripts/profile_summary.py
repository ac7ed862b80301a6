"""Condense a rocprofv3 kernel_stats.csv (+ the bench JSON line printed by the
same command) into a short text summary for profiles/.

  python scripts/profile_summary.py STATS.csv BENCH.log > profiles/X.txt"""
import csv
import json
import re
import sys

stats, log = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(stats)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"rocprofv3 --kernel-trace --stats  ({stats})")
print(f"{'kernel':58s} {'calls':>7s} {'avg_us':>9s} {'min_us':>8s} {'max_us':>8s} {'%':>6s}")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    n = re.sub(r"rst::\(anonymous namespace\)::", "", r["Name"])
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n)[:58]
    print(f"{n:58s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f} "
          f"{float(r['MinNs'])/1e3:8.2f} {float(r['MaxNs'])/1e3:8.2f} "
          f"{100*float(r['TotalDurationNs'])/tot:6.2f}")
for line in open(log):
    if line.startswith("{"):
        d = json.loads(line)
        rf = d["roofline"]
        print(f"\nsame command's bench line: value {d['value']:.1f} {d['unit']}, "
              f"{rf['kernel']} avg {rf['avg_us']:.2f} us (HIP events: {rf.get('timing', '')}), "
              f"achieved {rf['achieved']:.1f} GB/s = {100*rf['frac']:.2f}% of {rf['peak']} GB/s")
