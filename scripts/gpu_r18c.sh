#!/bin/bash
# the host API pair under the fallback's runtime knobs; the callers' pair with
# the small-cloud fallback off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for cfg in "X=0" "RST_LANE_MIN_DIV=2" "RST_LANE_MIN_DIV=1" "RST_LANE_MIN_FLOOR=1000000000" "X=1" "RST_LANE_MIN_DIV=2" "RST_LANE_MIN_DIV=1"; do
  env $cfg timeout -k 10 120 python tools/host_prof.py 4 > gpurun_out/r18c_host.txt 2>&1 || { tail -5 gpurun_out/r18c_host.txt; exit 1; }
  echo "$cfg: $(grep pair gpurun_out/r18c_host.txt | awk '{s+=$3} END {printf "%.2f ms avg over %d", s/NR, NR}')"
done
for cfg in "X=0" "RST_SMALL_FB_N=0" "X=1" "RST_SMALL_FB_N=0" "RST_LANE_MIN_FLOOR=1000000000"; do
  env $cfg timeout -k 10 120 python tools/callers_prof.py ref 4 > gpurun_out/r18c_callers.txt 2>&1 || { tail -5 gpurun_out/r18c_callers.txt; exit 1; }
  echo "callers $cfg: $(grep pair gpurun_out/r18c_callers.txt | awk '{print $(NF-4)}' | tr '\n' ' ')"
done
