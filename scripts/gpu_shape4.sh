#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for rep in 1 2; do
for cfg in "12 4" "16 4" "20 4"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps 20 --warmup 5 --batch $1 --inflight $2 > gpurun_out/shape4_$1_$2.log 2>&1 || { tail -5 gpurun_out/shape4_$1_$2.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/shape4_$1_$2.log').read().strip().splitlines()[-1]);print('rep $rep batch $1 inflight $2 value', round(d['value']), 'ok', d['pairs_ok'])"
done
done
