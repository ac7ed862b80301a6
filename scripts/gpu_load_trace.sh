#!/bin/bash
# Kernel trace of the loaded REF value leg (24 pairs in flight) and of one
# pair alone, then scripts/load_profile.py: launches/s, kernels at once,
# per-kernel durations under load vs alone.   TAG=x bash scripts/gpu_load_trace.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-load}
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --roof-steps 1 --no-host-api"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/load_${TAG} -o run -- python3 bench.py $B --steps ${STEPS:-48} ${EXTRA} > gpurun_out/${TAG}_load_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/solo_${TAG} -o run -- python3 bench.py $B --inflight 1 --steps 3 --warmup 1 ${EXTRA} > /dev/null 2>&1 || exit $?
python3 scripts/load_profile.py $(find gpurun_out/load_${TAG} -name "*kernel_trace.csv") $(find gpurun_out/solo_${TAG} -name "*kernel_trace.csv") > gpurun_out/${TAG}_load_profile.txt
tail -1 gpurun_out/${TAG}_load_bench.log | cut -c1-200
head -24 gpurun_out/${TAG}_load_profile.txt
