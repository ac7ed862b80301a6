#!/bin/bash
# Development round trip: GPU parity tests, the fallback anatomy (diag
# build), the default bench without the CPU legs, a one-pair iteration trace.
#   TAG=r02f bash scripts/gpu_dev.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here, not in bench.py
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-dev}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/${TAG}_$name.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_$name.log | head -20; exit $rc; }
}
step pytest_gpu 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread
step diag 200 env RST_LIB=realsensetracker_amd/lib/variants/diag.so python tools/diag_fb.py
cat gpurun_out/${TAG}_diag.log
step bench 400 python bench.py --no-cpu --no-host-api --no-gicp
step iter 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/iter_${TAG} -o run -- python3 bench.py --inflight 1 --steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0
python3 scripts/iter_profile.py $(find gpurun_out/iter_${TAG} -name "*kernel_trace.csv") > gpurun_out/${TAG}_iteration_profile.txt
cat gpurun_out/${TAG}_iteration_profile.txt
