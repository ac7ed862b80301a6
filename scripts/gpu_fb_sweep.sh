#!/bin/bash
# Sweep the fallback grid (RST_FB_BLOCKS) x pairs in flight on the default
# stream bench (no CPU baseline / extra modes).
#   FB="2048 1024 512" INFLIGHT="2 3" bash scripts/gpu_fb_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for fb in ${FB:-2048 1024 512 256}; do
  for k in ${INFLIGHT:-2 3}; do
    f=gpurun_out/sweep_fb${fb}_if$k.log
    RST_FB_BLOCKS=$fb timeout -k 10 300 python bench.py --no-cpu --no-p2plane --no-host-api --no-gicp --inflight $k ${EXTRA} > $f 2>&1 || exit $?
    echo "fb $fb inflight $k: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps k_icp_nn", round(d["roofline"]["avg_us"],1), "us")')"
  done
done
