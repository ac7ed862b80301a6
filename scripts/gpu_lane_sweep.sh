#!/bin/bash
# Sweep the fallback's lane-mode threshold (RST_LANE_MIN_DIV) on the stream
# and pyramid benches.
set -o pipefail
mkdir -p gpurun_out
for d in ${DIVS:-0 2 4 8 16}; do
  for wl in ${WORKLOADS:-stream pyramid}; do
    f=gpurun_out/lane_${d}_${wl}.log
    RST_LANE_MIN_DIV=$d timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-p2plane --no-host-api --no-gicp > $f 2>&1 || exit $?
    echo "div $d $wl: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps")')"
  done
done
