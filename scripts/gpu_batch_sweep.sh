#!/bin/bash
# The batched value leg: GPU tests of the batch, then value by (pairs per
# batch, batches in flight).   TAG=x bash scripts/gpu_batch_sweep.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-batch}
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --roof-steps 1 --no-host-api"
for cfg in ${CFGS:-"0 24" "8 2" "8 4" "12 2" "24 1" "24 2"}; do
  set -- $cfg
  timeout -k 10 300 python bench.py $B --batch $1 --inflight $2 --steps ${STEPS:-96} > gpurun_out/${TAG}_b$1_i$2.log 2>&1 || { tail -5 gpurun_out/${TAG}_b$1_i$2.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_b$1_i$2.log').read().strip().splitlines()[-1]);print('batch $1 inflight $2 value', round(d['value']), 'pairs_ok', d['pairs_ok'])"
done
