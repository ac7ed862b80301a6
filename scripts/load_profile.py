"""Concurrency of a loaded run from a rocprofv3 kernel trace: per kernel the
launches and mean duration under load, the wall span, the time any kernel
runs, and how many kernels run at once (time-weighted).

    python scripts/load_profile.py TRACE.csv [SOLO_TRACE.csv]

With a solo trace (one pair in flight) the per-kernel durations are set
side by side: a kernel slower under load shares something (CUs, L2, HBM);
one as fast leaves the chip idle while the pairs wait on each other.
"""
import csv
import re
import sys
from collections import defaultdict


def short(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1]


def load(path):
    rows = list(csv.DictReader(open(path)))
    ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    ev.sort(key=lambda e: e[1])
    return ev


def stats(ev):
    per = defaultdict(list)
    for n, s, e in ev:
        per[n].append((e - s) / 1000.0)
    return per


def main():
    ev = load(sys.argv[1])
    # the loop's steady part: drop the first and last 10% of the launches
    k = len(ev) // 10
    core = ev[k:len(ev) - k] if len(ev) > 20 else ev
    t0 = min(s for _, s, _ in core)
    t1 = max(e for _, _, e in core)
    span = (t1 - t0) / 1000.0
    # time-weighted number of kernels running at once
    pts = []
    for _, s, e in core:
        pts.append((s, 1))
        pts.append((e, -1))
    pts.sort()
    cur, last, busy, hist = 0, pts[0][0], 0, defaultdict(float)
    for t, d in pts:
        if t > last:
            hist[cur] += (t - last) / 1000.0
            if cur > 0:
                busy += (t - last) / 1000.0
        cur += d
        last = t
    tot = sum((e - s) / 1000.0 for _, s, e in core)
    print(f"launches {len(core)} over {span:.0f} us: {len(core) / span * 1e6:.0f} launches/s; "
          f"kernel time {tot:.0f} us = {tot / span:.2f} kernels at once on average, "
          f"{tot / max(busy, 1e-9):.2f} while any runs; GPU idle {100 * (1 - busy / span):.1f}%")
    print("kernels at once -> share of time: " +
          ", ".join(f"{c}: {100 * v / span:.1f}%" for c, v in sorted(hist.items()) if v / span > 0.005))
    per = stats(core)
    solo = stats(load(sys.argv[2])) if len(sys.argv) > 2 else {}
    print(f"{'kernel':<24}{'launches':>9}{'mean us':>10}{'solo us':>10}{'share':>8}")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        sm = sum(solo[n]) / len(solo[n]) if n in solo else float("nan")
        print(f"{n[:24]:<24}{len(d):>9}{sum(d) / len(d):>10.1f}{sm:>10.1f}{100 * sum(d) / tot:>7.1f}%")


if __name__ == "__main__":
    main()
