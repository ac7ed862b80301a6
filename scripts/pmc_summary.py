"""Average PMC counter values per kernel from rocprofv3 counter_collection.csv
files:  python scripts/pmc_summary.py gpurun_out/pmc_*/**/counter_collection.csv"""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("rst::(anonymous namespace)::", ""))[:40]
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n in sorted(acc, key=lambda k: -sum(acc[k].get("SQ_WAVE_CYCLES", [0]))):
    c = acc[n]
    print(n, " ".join(f"{k}={sum(v)/len(v):.4g}" for k, v in sorted(c.items())))
