#!/bin/bash
# the REF loop's 256-point ball chunks: GPU suite, every leg
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r14b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r14b_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r14b_tests.log | head -20; exit $rc; }
TAG=legs5 bash scripts/gpu_legs2.sh
