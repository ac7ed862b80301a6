#!/bin/bash
# fused covariance + solve for small clouds: GPU suite, callers profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r11l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r11l_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r11l_tests.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/callers_r11l -o run -- python3 tools/callers_prof.py ref 3 > gpurun_out/r11l_callers.log 2>&1 || exit 1
grep "pair" gpurun_out/r11l_callers.log | tail -3
python3 scripts/iter_profile_all.py $(find gpurun_out/callers_r11l -name "*kernel_trace.csv") > gpurun_out/r11l_callers_iteration_profile.txt
head -8 gpurun_out/r11l_callers_iteration_profile.txt | cut -c1-110; tail -2 gpurun_out/r11l_callers_iteration_profile.txt | cut -c1-300
