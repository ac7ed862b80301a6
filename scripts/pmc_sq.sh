#!/bin/bash
# One SQ counter pass over a short single-pair bench (kernel-1 instruction mix).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sq}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d gpurun_out/${TAG} -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-p2plane --no-host-api --inflight 1 > gpurun_out/${TAG}.log 2>&1
