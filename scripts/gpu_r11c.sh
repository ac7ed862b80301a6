#!/bin/bash
# iteration-0 pixel windows (16 / 20 / 24 px caps) behind sparse-ring seeds
set -o pipefail
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
TAG=r11c VARIANTS="s3i16 s3i20 s3i24" bash scripts/gpu_variants.sh
