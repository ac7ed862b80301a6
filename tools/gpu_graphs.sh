#!/bin/bash
# bench value with and without hipGraph replay of the iteration loop
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-graphs}
for g in "" "--graphs"; do
  for inf in $1; do
    timeout -k 10 300 python bench.py --steps 24 --warmup 6 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 --inflight $inf $g > gpurun_out/${TAG}_i${inf}$g.log 2>&1 || exit $?
    echo "inflight $inf $g: $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_i${inf}$g.log | head -1)"
  done
done
