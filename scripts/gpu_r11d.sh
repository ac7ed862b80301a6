#!/bin/bash
# group composites by whole-wavefront chains (gc1), reseed rings (r3)
set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
mkdir -p gpurun_out
RST_LIB=$PWD/realsensetracker_amd/lib/variants/gc1.so timeout -k 10 120 python tools/seqsum_stage.py 3 frame > gpurun_out/r11d_stage_gc1.txt 2>&1 || exit 1
grep -E "phases" gpurun_out/r11d_stage_gc1.txt
TAG=r11d VARIANTS="gc1 gc1s r3 s3i24r3" bash scripts/gpu_variants.sh
