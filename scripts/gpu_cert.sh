#!/bin/bash
# Far-point certificates: targeted GPU tests, full GPU suite, diag trace, A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "two_nearest or certificates or fallback or full_size" --timeout 120 --timeout-method thread > gpurun_out/cert_pytest.log 2>&1 || { tail -40 gpurun_out/cert_pytest.log; exit 1; }
tail -1 gpurun_out/cert_pytest.log
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cert_pytest_all.log 2>&1 || { tail -40 gpurun_out/cert_pytest_all.log; exit 1; }
tail -1 gpurun_out/cert_pytest_all.log
timeout -k 10 120 python scripts/diag_icp.py > gpurun_out/diag_cert.log 2>&1 || exit 1
grep "slow queue" gpurun_out/diag_cert.log | head -2 | cut -c1-400
VARIANTS="fb4" bash scripts/gpu_variant_ab.sh
