#!/bin/bash
# Quick GPU check: parity tests, ICP diag, bench (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python scripts/diag_icp.py > gpurun_out/diag.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log
