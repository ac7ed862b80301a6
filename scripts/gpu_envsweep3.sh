#!/bin/bash
# the fallback grid over every leg (env RST_FB_BLOCKS)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for fb in 384 128 96 64; do
  RST_FB_BLOCKS=$fb timeout -k 10 500 python bench.py --no-cpu --no-gicp > gpurun_out/env3_$fb.log 2>&1 || { tail -3 gpurun_out/env3_$fb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env3_$fb.log').read().strip().splitlines()[-1]);print('fb $fb value', round(d['value']), 'fp64', round(d['fp64_sums']['iterations_per_s']), 'p2plane', round(d['p2plane']['iterations_per_s']), 'knn', round(d['p2plane']['knn16_normals']['iterations_per_s']), 'host', round(d['host_api']['ms_per_pair'],2), 'callers', round(d['callers_workload']['ref_sums']['ms_per_pair'],2), round(d['callers_workload']['fp64_sums']['ms_per_pair'],2))"
  RST_FB_BLOCKS=$fb timeout -k 10 300 python bench.py --workload sharded --steps 5 --warmup 1 > gpurun_out/env3_sh_$fb.log 2>&1 || { tail -3 gpurun_out/env3_sh_$fb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env3_sh_$fb.log').read().strip().splitlines()[-1]);print('fb $fb sharded', round(d['value']))"
done
