#!/bin/bash
# A/B of library variants (lib/variants/V.so) on the batched value leg and a
# one-pair iteration profile (iteration 0 / cold start), after the batch and
# parity tests of each variant.  TAG=x VARIANTS="a b" [TESTS=...] bash scripts/gpu_variants.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-var}
TESTS=${TESTS:-tests/test_gpu_batch.py}
B="--no-cpu --no-p2plane --no-gicp --no-sharded --ref-steps 0 --no-host-api --steps 20 --warmup 5"
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  echo "== $V"
  RST_LIB=$LIBV timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_${V}_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${TAG}_${V}_tests.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_${V}_tests.log | head -30; exit $rc; }
  RST_LIB=$LIBV timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_${V}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_${V}_bench.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${V}_bench.log').read().strip().splitlines()[-1]);print('$V value', round(d['value']), 'ok', d['pairs_ok'], 'kernels', {k: round(v, 1) for k, v in d['roofline']['kernels_avg_us'].items()})"
  RST_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/iter_${TAG}_${V} -o run -- python3 bench.py --batch 0 --inflight 1 --steps 3 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --no-sharded --ref-steps 0 > gpurun_out/${TAG}_${V}_iter.log 2>&1 || { tail -5 gpurun_out/${TAG}_${V}_iter.log; exit 1; }
  python3 scripts/iter_profile_all.py $(find gpurun_out/iter_${TAG}_${V} -name "*kernel_trace.csv") > gpurun_out/${TAG}_${V}_iteration_profile.txt
  head -9 gpurun_out/${TAG}_${V}_iteration_profile.txt | cut -c1-170
  tail -2 gpurun_out/${TAG}_${V}_iteration_profile.txt | cut -c1-300
done
