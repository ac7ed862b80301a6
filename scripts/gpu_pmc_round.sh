#!/bin/bash
# Per-iteration kernel trace (one pair in flight) and PMC passes of the
# ICP loop's kernels on the default 640x480 stream, one counter group per
# rocprofv3 run (separate passes, hardware limits per block).
#   TAG=r02d bash scripts/gpu_pmc_round.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here, not in bench.py
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-pmc}
SHORT="--inflight 1 --steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --no-sharded --ref-steps 0 --roof-steps 0"
run() {  # name, limit, rocprof args...
  local name=$1 lim=$2; shift 2
  timeout -s KILL "$lim" rocprofv3 "$@" --output-format csv -d gpurun_out/${TAG}_$name -o run -- python3 bench.py $SHORT > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run trace 300 --kernel-trace
python3 scripts/iter_profile.py $(find gpurun_out/${TAG}_trace -name "*kernel_trace.csv") > gpurun_out/${TAG}_iteration_profile.txt
cat gpurun_out/${TAG}_iteration_profile.txt
run sq 120 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
run tcc 120 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
run fetch 120 --pmc FETCH_SIZE
run write 120 --pmc WRITE_SIZE
