#!/bin/bash
# the new defaults (20 / 24-pixel windows, batch 12): GPU suite + the driver's bench command
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r11j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r11j_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r11j_tests.log | head -20; exit $rc; }
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r11j_bench.log 2>&1 || { tail -5 gpurun_out/r11j_bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r11j_bench.log').read().strip().splitlines()[-1]);print('value', round(d['value']), 'frac', d['roofline']['frac'], 'fp64', round(d['fp64_sums']['iterations_per_s']), 'p2plane', round(d['p2plane']['iterations_per_s']), 'knn', round(d['p2plane']['knn16_normals']['iterations_per_s']), 'callers', {k: round(v['ms_per_pair'],2) for k, v in d['callers_workload'].items() if isinstance(v, dict) and 'ms_per_pair' in v}, 'host_api', round(d['host_api']['ms_per_pair'],2), 'cpu', d['cpu_baseline'])"
