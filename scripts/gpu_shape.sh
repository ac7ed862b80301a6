#!/bin/bash
# batch x in-flight sweep of the value leg (default library)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for cfg in "8 4" "8 5" "8 6" "12 3" "12 4" "16 2" "16 3" "6 6"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --no-cpu --no-p2plane --no-gicp --no-sharded --ref-steps 0 --no-host-api --steps 20 --warmup 5 --batch $1 --inflight $2 > gpurun_out/shape_$1_$2.log 2>&1 || { tail -5 gpurun_out/shape_$1_$2.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/shape_$1_$2.log').read().strip().splitlines()[-1]);print('batch $1 inflight $2 value', round(d['value']), 'ok', d['pairs_ok'])"
done
