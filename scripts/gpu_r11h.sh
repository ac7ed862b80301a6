#!/bin/bash
# k_icp_bf slices / queue threshold sweep on the callers' workload (REF)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for cfg in "0 16" "8 16" "8 32" "8 64" "4 64" "2 64" "16 64"; do
  set -- $cfg
  RST_BF_MIN_DIV=$1 RST_BF_SLICES=$2 timeout -k 10 120 python tools/callers_prof.py ref 4 > gpurun_out/r11h_$1_$2.log 2>&1 || exit 1
  echo "div $1 slices $2: $(grep 'pair' gpurun_out/r11h_$1_$2.log | tail -3 | sed 's/.*align/align/' | tr '\n' ' ')"
done
RST_BF_MIN_DIV=8 RST_BF_SLICES=64 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/callers_r11h -o run -- python3 tools/callers_prof.py ref 3 > gpurun_out/r11h_prof.log 2>&1 || exit 1
python3 scripts/iter_profile_all.py $(find gpurun_out/callers_r11h -name "*kernel_trace.csv") > gpurun_out/r11h_callers_iteration_profile.txt
head -14 gpurun_out/r11h_callers_iteration_profile.txt | cut -c1-100
