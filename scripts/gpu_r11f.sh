#!/bin/bash
# k_sq_small A/B: workgroups per chain (RST_SQ_SMALL_WG) x group composites
# (lane chains / whole-wavefront chains, smc0 variant)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for V in default smc0; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  for WG in 1 2 4; do
    echo "== $V wg $WG"
    RST_LIB=$LIBV RST_SQ_SMALL_WG=$WG timeout -k 10 120 python tools/small_stats.py > gpurun_out/r11f_${V}_${WG}.txt 2>&1 || exit 1
    grep -E "15k" gpurun_out/r11f_${V}_${WG}.txt | cut -c1-150
    RST_LIB=$LIBV RST_SQ_SMALL_WG=$WG timeout -k 10 120 python tools/callers_prof.py ref 3 > gpurun_out/r11f_${V}_${WG}_callers.txt 2>&1 || exit 1
    grep "pair" gpurun_out/r11f_${V}_${WG}_callers.txt | tail -3
  done
done
