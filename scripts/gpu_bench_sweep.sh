#!/bin/bash
# Bench sweep over pairs in flight x kernel-1 variants (no CPU baseline).
#   INFLIGHT="1 2" VARIANTS="0 1" bash scripts/gpu_bench_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-0}; do
  for k in ${INFLIGHT:-1 2}; do
    f=gpurun_out/bench_v${v}_if$k.log
    RST_NN_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu --no-p2plane --inflight $k > $f 2>&1 || exit $?
    echo "variant $v inflight $k: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps k_icp_nn", round(d["roofline"]["avg_us"],1), "us")')"
  done
done
