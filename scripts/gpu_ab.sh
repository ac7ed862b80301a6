#!/bin/bash
# A/B of library variants (lib/variants/*.so) on the REF value bench, the
# fp64 leg and a one-pair iteration profile.   VARIANTS="default x y" TAG=ab bash scripts/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-ab}
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --roof-steps 1"
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset RST_LIB; else export RST_LIB=realsensetracker_amd/lib/variants/$v.so; fi
  timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_$v.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/iter_${TAG}_$v -o run -- python3 bench.py $B --no-host-api --inflight 1 --steps 3 --warmup 1 > /dev/null 2>&1 || exit $?
  python3 scripts/iter_profile_all.py $(find gpurun_out/iter_${TAG}_$v -name "*kernel_trace.csv") > gpurun_out/${TAG}_${v}_iter.txt
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_$v.log').read().strip().splitlines()[-1]);print('$v value', round(d['value']), 'host_api ms', round(d['host_api']['ms_per_pair'],1), 'callers ref ms', round(d['callers_workload']['ref_sums']['ms_per_pair'],1))"
  sed -n 3,6p gpurun_out/${TAG}_${v}_iter.txt | cut -c1-120; tail -1 gpurun_out/${TAG}_${v}_iter.txt
done
