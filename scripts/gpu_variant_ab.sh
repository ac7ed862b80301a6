#!/bin/bash
# A/B of variant libraries (realsensetracker_amd/lib/variants/*.so, built
# with RST_DEFINES) against the default on the stream and pyramid benches.
#   VARIANTS="polar1" bash scripts/gpu_variant_ab.sh
set -o pipefail
mkdir -p gpurun_out
for v in default ${VARIANTS}; do
  lib=""
  [ "$v" != default ] && lib="$PWD/realsensetracker_amd/lib/variants/$v.so"
  for wl in ${WORKLOADS:-stream pyramid}; do
    f=gpurun_out/ab_${v}_${wl}.log
    RST_LIB=${lib:-$PWD/realsensetracker_amd/lib/librst_align.so} timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-p2plane --no-host-api --no-gicp > $f 2>&1 || exit $?
    echo "$v $wl: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps k_icp_nn", round(d["roofline"]["avg_us"],1), "us")')"
  done
done
