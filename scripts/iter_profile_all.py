"""Per-iteration kernel durations and wall spans of one-pair-in-flight ICP
runs, every kernel of the loop (both sum modes), from a rocprofv3 kernel
trace:  python scripts/iter_profile_all.py TRACE.csv"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1]


pairs, it, t0 = 0, -1, 0
per = defaultdict(lambda: defaultdict(float))  # it -> kernel -> us
span = defaultdict(float)
names = []
for r in rows:
    n = short(r["Kernel_Name"])
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if n == "k_init_state":
        it, t0 = 0, e
        pairs += 1
        continue
    if it < 0:
        continue
    if n not in names:
        names.append(n)
    per[it][n] += (e - s) / 1000
    if n == "k_reduce_solve":
        span[it] += (e - t0) / 1000
        t0 = e
        it += 1
names = [n for n in names if sum(per[i][n] for i in per) > 0]
print(f"pairs {pairs}; per-pair us per iteration (kernel durations; span = wall time "
      f"from the previous solve's end to this one's)")
print("iter " + " ".join(f"{n[:12]:>12}" for n in names) + "     span")
for i in list(range(0, 6)) + [16, 32, 64, 126, 127]:
    if i in per:
        print(f"{i:4d} " + " ".join(f"{per[i][n] / pairs:12.1f}" for n in names)
              + f" {span[i] / pairs:8.1f}")
tot = {n: sum(per[i][n] for i in per) / pairs for n in names}
print("per pair totals us: " + ", ".join(f"{n} {v:.0f}" for n, v in tot.items()))
print("kernel sum per pair us", round(sum(tot.values())), " wall span per pair us",
      round(sum(span.values()) / pairs))
