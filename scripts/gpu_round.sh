#!/bin/bash
# One GPU session: tests, smoke, bench, kernel-trace profile.  Every GPU step
# has its own time limit; the chain stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -5 gpurun_out/$name.log
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu
find gpurun_out/prof_${TAG} -name "*stats*"
