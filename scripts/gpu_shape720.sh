#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for b in 6 8 12; do
  timeout -k 10 400 python bench.py --width 1280 --height 720 --no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps 20 --warmup 5 --batch $b > gpurun_out/s720_$b.log 2>&1 || { tail -5 gpurun_out/s720_$b.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/s720_$b.log').read().strip().splitlines()[-1]);print('720p batch $b value', round(d['value']), 'ok', d['pairs_ok'])"
done
