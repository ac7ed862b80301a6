#!/bin/bash
# One GPU round trip of the build/measure loop: parity tests, the default
# bench, and a per-iteration kernel trace (one pair in flight).
#   TAG=r02b bash scripts/gpu_iter.sh [--no-tests]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/${TAG}_$name.log
  [ $rc -eq 0 ] || exit $rc
}
if [ "$1" != "--no-tests" ]; then
  step pytest_gpu 600 python -u -m pytest tests/ -q -s -rf -m gpu --maxfail=10 --timeout 300 --timeout-method thread
fi
step bench 400 python bench.py --steps 20 --warmup 5
step iter 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/iter_${TAG} -o run -- python3 bench.py --inflight 1 --steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0
python3 scripts/iter_profile.py $(find gpurun_out/iter_${TAG} -name "*kernel_trace.csv") > gpurun_out/${TAG}_iteration_profile.txt
cat gpurun_out/${TAG}_iteration_profile.txt
