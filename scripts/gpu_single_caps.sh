#!/bin/bash
# A/B of a lone align's window caps (RST_PIX_HALF_SINGLE / RST_ROW_HALF_SINGLE
# variants): host API, the callers' workload, the pyramid, and a short value
# leg.  TAG=x VARIANTS="a b" bash scripts/gpu_single_caps.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
TAG=${TAG:-caps}
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  RST_LIB=$LIBV timeout -k 10 400 python bench.py --no-cpu --no-gicp --no-sharded --no-p2plane --ref-steps 0 --steps 5 --warmup 2 > gpurun_out/${TAG}_${V}.log 2>&1 || { tail -3 gpurun_out/${TAG}_${V}.log; exit 1; }
  RST_LIB=$LIBV timeout -k 10 300 python bench.py --workload pyramid --graphs --no-p2plane --steps 48 > gpurun_out/${TAG}_${V}_pyr.log 2>&1 || { tail -3 gpurun_out/${TAG}_${V}_pyr.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${V}.log').read().strip().splitlines()[-1]);p=json.loads(open('gpurun_out/${TAG}_${V}_pyr.log').read().strip().splitlines()[-1]);print('$V value', round(d['value']), 'host', round(d['host_api']['ms_per_pair'],2), 'callers', round(d['callers_workload']['ref_sums']['ms_per_pair'],2), round(d['callers_workload']['fp64_sums']['ms_per_pair'],2), 'pyramid', round(p['value']))"
done
