#!/bin/bash
# Round-end evidence on one GPU: parity tests, smoke, default bench (with the
# CPU baseline), kernel-trace stats of a short bench, two PMC passes for the
# HBM traffic of k_icp_nn.  Each GPU step has its own limit; the chain stops
# at the first failure.   TAG=r01d bash scripts/gpu_profile_round.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here, not in bench.py
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-r01}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/${TAG}_$name.log
  [ $rc -eq 0 ] || exit $rc
}
SHORT="--steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --no-sharded"
step pytest_gpu 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
# the default bench command again under the tracer: its own JSON line
# (roofline.avg_us from HIP events) next to rocprof's per-kernel averages
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG} -o run -- python3 bench.py $SHORT
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_${TAG} -o run -- python3 bench.py $SHORT
python3 scripts/pmc_traffic.py gpurun_out/pmc_${TAG}.json $(find gpurun_out/pmcf_${TAG} -name "*counter_collection.csv") $(find gpurun_out/pmcw_${TAG} -name "*counter_collection.csv")
find gpurun_out/prof_${TAG} -name "*stats*"
