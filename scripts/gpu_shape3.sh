#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for cfg in "12 4 40" "16 4 30" "12 5 40" "16 3 30" "20 3 24" "24 2 20"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps $3 --warmup 5 --batch $1 --inflight $2 > gpurun_out/shape3_$1_$2.log 2>&1 || { tail -5 gpurun_out/shape3_$1_$2.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/shape3_$1_$2.log').read().strip().splitlines()[-1]);print('batch $1 inflight $2 steps $3 value', round(d['value']), 'ok', d['pairs_ok'])"
done
