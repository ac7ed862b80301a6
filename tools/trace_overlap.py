"""How the batched ICP loop's kernels share the GPU, from a rocprofv3 kernel
trace of the value bench: per loop kernel its mean duration and how many
other loop kernels ran beside it, per queue the fraction of the window its
kernels were running and the mean gap between one kernel's end and the
next one's start, and over the window how long 0, 1, 2, ... loop kernels
were resident at once.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- \\
        python3 bench.py --no-cpu --no-p2plane --no-gicp --ref-steps 0 \\
        --roof-steps 1 --no-host-api --steps 48
    python tools/trace_overlap.py gpurun_out/tr/run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("rst::", "")
    m = re.search(r"(k_\w+?)(<[^>(]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                     short(r["Kernel_Name"])))
loop = [r for r in rows if re.search(r"_b(<|$)", r[3])]
if not loop:
    sys.exit("no batched loop kernels in the trace")
loop.sort()
# the steady window: from the 10th percentile of starts to the 90th of ends
st = np.array([r[0] for r in loop])
en = np.array([r[1] for r in loop])
t0, t1 = np.percentile(st, 10), np.percentile(en, 90)
win = [r for r in loop if r[0] >= t0 and r[1] <= t1]
span = t1 - t0
print(f"window {span / 1e3:.0f} us, {len(win)} loop kernels, queues {sorted({r[2] for r in win})}")

# residency histogram over the window
ev = sorted([(r[0], 1) for r in win] + [(r[1], -1) for r in win])
hist = defaultdict(float)
cur, last = 0, t0
for t, d in ev:
    hist[cur] += t - last
    cur += d
    last = t
hist[cur] += t1 - last
print("loop kernels resident at once (share of the window):",
      {k: round(v / span, 3) for k, v in sorted(hist.items())})

# per kernel: duration and overlap with other loop kernels
per = defaultdict(list)
for i, (s, e, q, n) in enumerate(win):
    others = sum(1 for (s2, e2, q2, n2) in win if q2 != q and s2 < e and e2 > s)
    per[n].append((e - s, others))
print(f"{'kernel':28s} {'count':>5s} {'mean us':>8s} {'p90 us':>8s} {'others at once':>14s}")
tot = 0.0
for n, v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    d = np.array([x[0] for x in v]) / 1e3
    o = np.mean([x[1] for x in v])
    tot += d.sum()
    print(f"{n:28s} {len(v):5d} {d.mean():8.1f} {np.percentile(d, 90):8.1f} {o:14.2f}")
print(f"sum of loop kernel durations / window = {tot * 1e3 / span:.2f}")

# per queue: busy fraction and gaps
byq = defaultdict(list)
for r in win:
    byq[r[2]].append(r)
for q, v in sorted(byq.items()):
    v.sort()
    busy = sum(e - s for s, e, _, _ in v)
    gaps = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
    g = np.array(gaps) / 1e3
    after = defaultdict(list)
    for i in range(len(v) - 1):
        after[v[i][3]].append(g[i])
    print(f"queue {q}: busy {busy / span:.2f}, gap mean {g.mean():.1f} us p50 {np.median(g):.1f} "
          f"p90 {np.percentile(g, 90):.1f}; mean gap after: "
          + ", ".join(f"{k} {np.mean(x):.1f}" for k, x in sorted(after.items())))
