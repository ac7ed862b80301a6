#!/bin/bash
# Build-measure round trip on one GPU: the named test files first (fast
# fail), then the whole -m gpu suite, then the default bench.  Each GPU step
# has its own limit; the chain stops at the first failure.
#   TAG=r02b bash scripts/gpu_check.sh tests/test_gpu_seqsum.py
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-chk}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 gpurun_out/${TAG}_$name.log
  [ $rc -eq 0 ] || exit $rc
}
if [ $# -gt 0 ]; then
  step first 300 python -u -m pytest "$@" -x -v -s -m gpu --timeout 120 --timeout-method thread
fi
[ -n "$NO_SUITE" ] || step pytest_gpu 600 python -u -m pytest tests/ -q -rf -m gpu --maxfail=5 --timeout 300 --timeout-method thread
[ -n "$NO_BENCH" ] || step bench 400 python bench.py
