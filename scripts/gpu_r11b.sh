#!/bin/bash
# iteration-0 pixel windows behind sparse-ring seeds (variants), the map
# kernel's phase clocks on a frame, in-flight depth A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 120 python tools/seqsum_stage.py 3 frame > gpurun_out/r11b_stage.txt 2>&1 || exit 1
grep -E "phases|status" gpurun_out/r11b_stage.txt
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps 20 --warmup 5"
for IF in 3 6; do
  timeout -k 10 300 python bench.py $B --inflight $IF > gpurun_out/r11b_if$IF.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r11b_if$IF.log').read().strip().splitlines()[-1]);print('inflight $IF value', round(d['value']))"
done
TAG=r11b VARIANTS="s3i8 s3i12" bash scripts/gpu_variants.sh
