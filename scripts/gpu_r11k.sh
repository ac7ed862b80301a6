#!/bin/bash
# sharded aligns with the narrow window caps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "shard or comm or rccl or relay" --timeout 300 --timeout-method thread > gpurun_out/r11k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r11k_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r11k_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload sharded --steps 5 --warmup 1 > gpurun_out/r11k_sharded.log 2>&1 || { tail -5 gpurun_out/r11k_sharded.log; exit 1; }
timeout -k 10 300 python bench.py --workload sharded --steps 5 --warmup 1 --sum-mode fp64 > gpurun_out/r11k_sharded_fp64.log 2>&1 || { tail -5 gpurun_out/r11k_sharded_fp64.log; exit 1; }
for f in sharded sharded_fp64; do python3 -c "import json;d=json.loads(open('gpurun_out/r11k_$f.log').read().strip().splitlines()[-1]);print('$f', round(d['value']))"; done
