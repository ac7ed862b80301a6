#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps 20 --warmup 5"
for rep in 1 2; do
for fb in 96 64 48 32; do
  RST_FB_BLOCKS_BATCH=$fb timeout -k 10 300 python bench.py $B > gpurun_out/env4_$fb.log 2>&1 || { tail -3 gpurun_out/env4_$fb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env4_$fb.log').read().strip().splitlines()[-1]);print('fbb $fb value', round(d['value']), 'ok', d['pairs_ok'])"
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/env4_tests.log 2>&1; echo "batch tests rc=$?"; tail -1 gpurun_out/env4_tests.log
