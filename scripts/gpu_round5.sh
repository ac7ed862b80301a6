#!/bin/bash
# Round-5 development pass: parity tests (FIRST, then the whole suite), the
# driver's exact bench command, a kernel-trace of the reference callers'
# workload (per-iteration kernels at ~15k points) and rocprof stats of the
# bench.   TAG=r10b [FIRST=...] [SKIP_TESTS=1] bash scripts/gpu_round5.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-dev}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/${TAG}_$name.log | cut -c1-600
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_$name.log | head -20; exit $rc; }
}
if [ -n "$FIRST" ]; then
  step first 600 python -u -m pytest $FIRST -x -v -m gpu --timeout 300 --timeout-method thread
fi
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread
fi
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step callers 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/callers_${TAG} -o run -- python3 tools/callers_prof.py ref 3
python3 scripts/iter_profile_all.py $(find gpurun_out/callers_${TAG} -name "*kernel_trace.csv") > gpurun_out/${TAG}_callers_iteration_profile.txt
cat gpurun_out/${TAG}_callers_iteration_profile.txt | tail -8 | cut -c1-400
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-host-api --no-gicp --no-p2plane
python3 scripts/profile_summary.py $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv") gpurun_out/${TAG}_prof.log > gpurun_out/${TAG}_profile_summary.txt
head -30 gpurun_out/${TAG}_profile_summary.txt
