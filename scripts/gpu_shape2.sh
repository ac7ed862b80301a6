#!/bin/bash
# batch x in-flight on the same 480 pairs, and 12 x 4 / 12 x 5 at the driver's 20 steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for cfg in "8 4 60" "12 4 40" "10 4 48" "16 3 30" "12 5 20" "12 4 20"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps $3 --warmup 5 --batch $1 --inflight $2 > gpurun_out/shape2_$1_$2_$3.log 2>&1 || { tail -5 gpurun_out/shape2_$1_$2_$3.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/shape2_$1_$2_$3.log').read().strip().splitlines()[-1]);print('batch $1 inflight $2 steps $3 value', round(d['value']), 'ok', d['pairs_ok'])"
done
