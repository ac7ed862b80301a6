#!/bin/bash
# k_sq_small over up to 4 workgroups per chain: seqsum + callers parity,
# phase clocks, the callers' per-iteration profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 600 python -u -m pytest tests/test_gpu_seqsum.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "small or callers or seq or inloop" -s > gpurun_out/r11e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r11e_tests.log; grep "seq sums of" gpurun_out/r11e_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r11e_tests.log | head; exit $rc; }
timeout -k 10 120 python tools/small_stats.py > gpurun_out/r11e_small_stats.txt 2>&1 || exit 1
cat gpurun_out/r11e_small_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/callers_r11e -o run -- python3 tools/callers_prof.py ref 3 > gpurun_out/r11e_callers.log 2>&1 || exit 1
grep "pair" gpurun_out/r11e_callers.log | tail -3
python3 scripts/iter_profile_all.py $(find gpurun_out/callers_r11e -name "*kernel_trace.csv") > gpurun_out/r11e_callers_iteration_profile.txt
head -8 gpurun_out/r11e_callers_iteration_profile.txt | cut -c1-110; tail -2 gpurun_out/r11e_callers_iteration_profile.txt | cut -c1-300
