#!/bin/bash
# Stream bench over pairs in flight x HIP hardware queues (no CPU legs).
#   SWEEP="4:8 6:8 8:16" bash scripts/gpu_inflight_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for c in ${SWEEP:-4:24 6:24 8:24}; do
  inf=${c%%:*}; hq=${c#*:}
  f=gpurun_out/sweep_${inf}_${hq}.log
  timeout -k 10 300 python bench.py --inflight $inf --hw-queues $hq --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 $EXTRA > $f 2>&1 || exit $?
  echo "inflight $inf hwq $hq: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps")')"
done
