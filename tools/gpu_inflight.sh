#!/bin/bash
# bench value vs pairs in flight (and HIP hardware queues per process):
#   TAG=x bash tools/gpu_inflight.sh "2 3 4" "4 8"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-inflight}
for q in $2; do
  for inf in $1; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 24 --warmup 6 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 --inflight $inf > gpurun_out/${TAG}_q${q}_i${inf}.log 2>&1 || exit $?
    echo "queues $q inflight $inf: $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_q${q}_i${inf}.log | head -1)"
  done
done
