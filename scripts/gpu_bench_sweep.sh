#!/bin/bash
# Bench sweep over pairs in flight (no CPU baseline / extra modes).
#   INFLIGHT="1 2 3" EXTRA="--graphs" bash scripts/gpu_bench_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for k in ${INFLIGHT:-1 2}; do
  f=gpurun_out/bench_if$k${TAGX}.log
  timeout -k 10 300 python bench.py --no-cpu --no-p2plane --no-host-api --no-gicp --inflight $k $EXTRA > $f 2>&1 || exit $?
  echo "inflight $k $EXTRA: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps k_icp_nn", round(d["roofline"]["avg_us"],1), "us")')"
done
