#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps 20 --warmup 5"
for rep in 1 2; do
for fb in 384 256 192 128; do
  RST_FB_BLOCKS=$fb timeout -k 10 300 python bench.py $B > gpurun_out/env2_$fb.log 2>&1 || { tail -3 gpurun_out/env2_$fb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env2_$fb.log').read().strip().splitlines()[-1]);print('fb $fb value', round(d['value']), 'ok', d['pairs_ok'])"
done
done
for fb in 384 256; do
  RST_FB_BLOCKS=$fb timeout -k 10 400 python bench.py --no-cpu --no-host-api --no-gicp > gpurun_out/env2_legs_$fb.log 2>&1 || { tail -3 gpurun_out/env2_legs_$fb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env2_legs_$fb.log').read().strip().splitlines()[-1]);print('fb $fb legs value', round(d['value']), 'fp64', round(d['fp64_sums']['iterations_per_s']), 'p2plane', round(d['p2plane']['iterations_per_s']), 'knn', round(d['p2plane']['knn16_normals']['iterations_per_s']))"
done
