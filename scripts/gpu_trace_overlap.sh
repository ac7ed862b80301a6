#!/bin/bash
# Kernel trace of the batched value bench and its overlap analysis
# (tools/trace_overlap.py).   TAG=x [GPU_MAX_HW_QUEUES=4] bash scripts/gpu_trace_overlap.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-tro}
B="bench.py --no-cpu --no-p2plane --no-gicp --ref-steps 0 --roof-steps 1 --no-host-api --steps ${STEPS:-48} ${EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tr -o run -- python3 $B > gpurun_out/${TAG}_tr.log 2>&1 || { tail -5 gpurun_out/${TAG}_tr.log; exit 1; }
tail -1 gpurun_out/${TAG}_tr.log | cut -c1-200
python3 tools/trace_overlap.py $(find gpurun_out/${TAG}_tr -name "*kernel_trace.csv") > gpurun_out/${TAG}_overlap.txt 2>&1
cat gpurun_out/${TAG}_overlap.txt
