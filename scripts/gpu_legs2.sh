#!/bin/bash
# every leg of the bench (host API, callers included) + the sharded pair, per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
TAG=${TAG:-legs2}
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  RST_LIB=$LIBV timeout -k 10 500 python bench.py --no-cpu --no-gicp --no-sharded > gpurun_out/${TAG}_${V}.log 2>&1 || { tail -3 gpurun_out/${TAG}_${V}.log; exit 1; }
  RST_LIB=$LIBV timeout -k 10 300 python bench.py --workload sharded --steps 5 --warmup 1 > gpurun_out/${TAG}_${V}_sh.log 2>&1 || { tail -3 gpurun_out/${TAG}_${V}_sh.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${V}.log').read().strip().splitlines()[-1]);s=json.loads(open('gpurun_out/${TAG}_${V}_sh.log').read().strip().splitlines()[-1]);print('$V value', round(d['value']), 'fp64', round(d['fp64_sums']['iterations_per_s']), 'p2plane', round(d['p2plane']['iterations_per_s']), 'knn', round(d['p2plane']['knn16_normals']['iterations_per_s']), 'host', round(d['host_api']['ms_per_pair'],2), 'callers', round(d['callers_workload']['ref_sums']['ms_per_pair'],2), round(d['callers_workload']['fp64_sums']['ms_per_pair'],2), 'sharded', round(s['value']))"
done
