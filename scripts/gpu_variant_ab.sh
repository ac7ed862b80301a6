#!/bin/bash
# Parity of library variants (lib/variants/V.so) on the value's own tests,
# then the value A/B (scripts/gpu_ab.sh).
#   TAG=x VARIANTS="a b" [TESTS="tests/test_gpu_batch.py"] bash scripts/gpu_variant_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-vab}
TESTS=${TESTS:-tests/test_gpu_batch.py tests/test_gpu_configs.py}
for V in ${TEST_DEFAULT:+default} ${NO_VARIANT_TESTS:-${VARIANTS}}; do
  [ "$V" = 1 ] && continue
  LIBV=$PWD/realsensetracker_amd/lib/variants/$V.so; [ "$V" = default ] && LIBV=""
  RST_LIB=$LIBV timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_${V}_tests.log 2>&1
  rc=$?; echo "$V tests rc=$rc"; tail -2 gpurun_out/${TAG}_${V}_tests.log
  [ $rc -eq 0 ] || exit $rc
done
TAG=$TAG VARIANTS="$VARIANTS" bash scripts/gpu_ab.sh
