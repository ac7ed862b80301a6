#!/bin/bash
# GPU parity tests + bench lines of the other BASELINE configs (720p stream,
# pyramid, sharded 1M pair).  Each GPU step has its own limit; the chain
# stops at the first failure.   TAG=r01g bash scripts/gpu_configs.sh
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
[ -n "$SKIP_TESTS" ] || step pytest_gpu 600 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread
# PMC passes (FETCH / WRITE, batched NN kernels) of the 720p reference loop and
# the 640x480 point-to-plane stream, before their bench lines (which read them)
PMCB="--steps 6 --warmup 1 --batch 8 --inflight 1 --no-cpu --no-p2plane --no-host-api --no-gicp --no-sharded --ref-steps 0"
pmc() {  # key, Acc, bench args...
  local key=$1 acc=$2; shift 2
  step pmcf_$key 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_${TAG}_$key -o run -- python3 bench.py $PMCB "$@"
  step pmcw_$key 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_${TAG}_$key -o run -- python3 bench.py $PMCB "$@"
  python3 scripts/pmc_traffic.py gpurun_out/pmc_${TAG}_$key.json $(find gpurun_out/pmcf_${TAG}_$key -name "*counter_collection.csv") $(find gpurun_out/pmcw_${TAG}_$key -name "*counter_collection.csv") $acc 8 $key
  cp gpurun_out/pmc_${TAG}_$key.json profiles/pmc_${TAG}_$key.json
  rm -rf gpurun_out/pmcf_${TAG}_$key gpurun_out/pmcw_${TAG}_$key  # (gpurun copies back <= 64 MiB)
}
pmc stream_1280x720_p2point_ref RefAcc --width 1280 --height 720
pmc stream_640x480_p2plane P2PlaneAcc --mode p2plane
step bench_pyramid 300 python bench.py --workload pyramid --graphs --no-p2plane --steps 96
step bench_sharded 300 python bench.py --workload sharded --steps 5 --warmup 1
step bench_sharded_fp64 300 python bench.py --workload sharded --steps 5 --warmup 1 --sum-mode fp64
step bench_sharded_p2plane 300 python bench.py --workload sharded --steps 5 --warmup 1 --mode p2plane
step bench_720p 300 python bench.py --width 1280 --height 720 --no-host-api --no-gicp --no-sharded
step bench_720p_p2plane 300 python bench.py --width 1280 --height 720 --mode p2plane --no-host-api --no-gicp --no-sharded
step bench_p2plane 300 python bench.py --mode p2plane --no-host-api --no-gicp --no-sharded
