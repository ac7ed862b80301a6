#!/bin/bash
# the bench's side legs (fp64 sums, point-to-plane + kNN normals) per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
TAG=${TAG:-legs}
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  RST_LIB=$LIBV timeout -k 10 400 python bench.py --no-cpu --no-host-api --no-gicp > gpurun_out/${TAG}_${V}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${V}.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${V}.log').read().strip().splitlines()[-1]);print('$V value', round(d['value']), 'fp64', round(d['fp64_sums']['iterations_per_s']), 'p2plane', round(d['p2plane']['iterations_per_s']), 'knn', round(d['p2plane']['knn16_normals']['iterations_per_s']))"
done
