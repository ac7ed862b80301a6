#!/bin/bash
# Development check of a change to the loop kernels: the whole GPU suite,
# the batched value bench, and (optionally) the fallback anatomy of a few
# bench pairs with the diagnostics build.   TAG=x DIAG="1 12" bash scripts/gpu_dev_full.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-dfull}
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_gpu.log | head -30; exit $rc; }
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --roof-steps 1 --no-host-api --batch 8 --inflight 4 --steps 96"
timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench.log').read().strip().splitlines()[-1]);print('value', round(d['value']), 'ok', d['pairs_ok'], 'kernels', {k: round(v, 1) for k, v in d['roofline']['kernels_avg_us'].items()})"
for k in ${DIAG}; do
  RST_LIB=realsensetracker_amd/lib/variants/diag.so timeout -k 10 100 python tools/diag_fb.py --bench-pair $k --ref > gpurun_out/${TAG}_diag_$k.txt 2>&1 || exit 1
done
