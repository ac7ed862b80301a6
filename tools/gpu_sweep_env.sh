#!/bin/bash
# Per-iteration kernel profile (one pair in flight) of the default library
# under each environment setting given ("NAME=V,NAME2=V2" per setting):
#   TAG=x bash tools/gpu_sweep_env.sh RST_LANE_MIN_DIV=3 "RST_LANE_MIN_DIV=4,RST_FB_BLOCKS=2048"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sweep}
B="bench.py --inflight 1 --steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0"
k=0
for v in "$@"; do
  k=$((k+1))
  ENVS=$(echo "$v" | tr ',' ' ')
  env $ENVS timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 > gpurun_out/${TAG}_${k}_bench.log 2>&1 || exit $?
  echo "== $v: $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_${k}_bench.log | head -1)"
done
