#!/bin/bash
# RST_SUM_REF as the value leg: bench line, rocprof kernel stats of the same
# command, and a one-pair-in-flight iteration trace.
#   TAG=r03b bash scripts/gpu_ref_prof.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-dev}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 gpurun_out/${TAG}_$name.log | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc
}
Q="--no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 --roof-steps 1"
step bench 300 python bench.py --sum-mode ref $Q --steps 48
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --sum-mode ref $Q --steps 48
step iter 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/iter_${TAG} -o run -- python3 bench.py --sum-mode ref $Q --inflight 1 --steps 3 --warmup 1
python3 scripts/iter_profile_all.py $(find gpurun_out/iter_${TAG} -name "*kernel_trace.csv") > gpurun_out/${TAG}_iteration_profile.txt
cat gpurun_out/${TAG}_iteration_profile.txt
python3 scripts/profile_summary.py $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv") gpurun_out/${TAG}_prof.log > gpurun_out/${TAG}_profile_summary.txt; cat gpurun_out/${TAG}_profile_summary.txt
