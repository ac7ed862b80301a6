#!/bin/bash
# Per-kernel register / LDS / scratch usage of one source (compile only).
#   bash scripts/kres.sh icp.hip [kernel-name-regex]
cd "$(dirname "$0")/../realsensetracker_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 --cuda-device-only \
  -I../../include -I. -c "$1" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys, subprocess
pat = re.compile(sys.argv[1])
cur = None; rec = {}
def flush():
    if cur and pat.search(cur):
        print(f"{cur[:60]:60s} " + " ".join(f"{k}={v}" for k, v in rec.items()))
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        flush()
        n = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = re.sub(r"rst::\(anonymous namespace\)::", "", n); cur = re.sub(r"^void ", "", cur); cur = re.sub(r"\(.*", "", cur); rec = {}
        continue
    m = re.search(r"remark: +([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and m.group(1) in ("VGPRs", "AGPRs", "ScratchSize", "Occupancy", "LDS Size"):
        rec[m.group(1).replace(" ", "")] = m.group(2)
flush()
' "${2:-.}"
