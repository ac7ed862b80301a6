#!/bin/bash
# the pyramid line against the single-align fallback grid (env RST_FB_BLOCKS)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for fb in 384 192 768; do
  RST_FB_BLOCKS=$fb timeout -k 10 400 python bench.py --workload pyramid --graphs --no-p2plane --no-cpu --steps 96 > gpurun_out/pyr_$fb.log 2>&1 || { tail -3 gpurun_out/pyr_$fb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/pyr_$fb.log').read().strip().splitlines()[-1]);print('pyr fb $fb value', round(d['value']), 'fps', round(d['frames_per_s'],1))"
done
