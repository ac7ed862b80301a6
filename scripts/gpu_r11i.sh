#!/bin/bash
# iteration-0 neighbours by source tile (k_icp_pre): GPU suite, A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r11i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r11i_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r11i_tests.log | head -20; exit $rc; }
TAG=r11i VARIANTS="pre0 pre24" TESTS=tests/test_gpu_batch.py bash scripts/gpu_variants.sh
