#!/bin/bash
# Two SQ counter passes (one pair in flight, short bench) and their per-kernel
# averages.   TAG=r02i bash scripts/gpu_pmc_sq.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here, not in bench.py
export GPU_MAX_HW_QUEUES=24
TAG=${TAG:-sq}
B="bench.py --steps 3 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --no-sharded --ref-steps 0 --inflight 1 ${EXTRA:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d gpurun_out/${TAG}_sq1 -o run -- python3 $B > gpurun_out/${TAG}_sq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- python3 $B > gpurun_out/${TAG}_sq2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $(find gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2 -name "*counter_collection.csv") > gpurun_out/${TAG}_pmc.txt
cat gpurun_out/${TAG}_pmc.txt
