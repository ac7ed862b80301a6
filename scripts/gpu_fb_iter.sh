#!/bin/bash
# Per-iteration k_icp_nn_b / k_icp_fb_b durations of one batch (the first
# 8 pairs), default library vs variants.   TAG=x VARIANTS="a" bash scripts/gpu_fb_iter.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-fbit}
B="--no-cpu --no-p2plane --no-gicp --no-sharded --ref-steps 0 --roof-steps 1 --no-host-api --batch 8 --inflight 1 --steps 8 --warmup 1"
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  RST_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fbit_${TAG}_$V -o run -- python3 bench.py $B > /dev/null 2>&1 || exit 1
  python3 - <<PY
import csv, glob, re, numpy as np
f = glob.glob("gpurun_out/fbit_${TAG}_$V/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
def nm(r): return re.sub(r"\(.*", "", r["Kernel_Name"].replace("rst::(anonymous namespace)::", "").replace("void ", ""))
for k in sorted({nm(r) for r in rows if re.search(r"_b(<|$)", nm(r))}) if "${ALLK:-}" else ("k_icp_nn_b<RefAcc>", "k_icp_fb_b<RefAcc>"):
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if nm(r) == k])
    d = d[-128:]  # the last align: the roofline pass's batch
    print("$V", k, "total", round(d.sum()), "it 0-7", [round(x) for x in d[:8]], "8-31", round(d[8:32].mean(), 1), "32-127", round(d[32:].mean(), 1))
PY
done
