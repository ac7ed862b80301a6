#!/bin/bash
# Development loop on the GPU box: the sequential-sum and full-size config
# tests (bit-exact in-loop traces), then the REF value bench A/B of the
# current library against lib/variants/$VARIANTS.
#   TAG=x VARIANTS="default r05" TESTS="tests/test_gpu_seqsum.py tests/test_gpu_configs.py" bash scripts/gpu_dev_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dev}
TESTS=${TESTS:-tests/test_gpu_seqsum.py tests/test_gpu_configs.py}
if [ "$TESTS" != none ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
fi
TAG=$TAG VARIANTS="${VARIANTS:-default}" bash scripts/gpu_ab.sh
