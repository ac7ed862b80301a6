#!/bin/bash
# Development loop for a seqsum change: the walk statistics of a hard pair,
# the map kernel's phase clocks, the sequential-sum and batch tests, and the
# batched value bench -- for the default library and each variant under
# lib/variants (VARIANTS="a b").   TAG=x VARIANTS="gchain" bash scripts/gpu_dev_variant.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-dvar}
B="--no-cpu --no-p2plane --no-gicp --no-sharded --ref-steps 0 --roof-steps 1 --no-host-api --batch 8 --inflight 4 --steps 96"
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  echo "== $V"
  RST_LIB=$LIBV timeout -k 10 300 python -u -m pytest tests/test_gpu_seqsum.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_${V}_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${TAG}_${V}_tests.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_${V}_tests.log | head -30; exit $rc; }
  RST_LIB=$LIBV timeout -k 10 120 python tools/seqsum_stage.py 3 frame > gpurun_out/${TAG}_${V}_stage.txt 2>&1 || exit 1
  grep "phases" gpurun_out/${TAG}_${V}_stage.txt
  RST_LIB=$LIBV timeout -k 10 300 python tools/walk_stats.py --first 14 --pairs 1 > gpurun_out/${TAG}_${V}_walk14.txt 2>&1 || exit 1
  grep -A3 "descent phases" gpurun_out/${TAG}_${V}_walk14.txt | tail -2
  RST_LIB=$LIBV timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_${V}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_${V}_bench.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${V}_bench.log').read().strip().splitlines()[-1]);print('$V value', round(d['value']), 'ok', d['pairs_ok'], 'kernels', {k: round(v, 1) for k, v in d['roofline']['kernels_avg_us'].items()})"
done
