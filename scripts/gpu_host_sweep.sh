#!/bin/bash
# the reference-shaped host API (one large pair alone) against the single-align fallback grid
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
for fb in 384 768 1024 1536; do
  RST_FB_BLOCKS=$fb timeout -k 10 200 python tools/host_api_prof.py > gpurun_out/host_$fb.log 2>&1 || { tail -3 gpurun_out/host_$fb.log; exit 1; }
  echo "fb $fb: $(grep pair gpurun_out/host_$fb.log | tr '\n' ' ')"
  RST_FB_BLOCKS=$fb timeout -k 10 300 python bench.py --workload sharded --steps 5 --warmup 1 > gpurun_out/host_sh_$fb.log 2>&1 || { tail -3 gpurun_out/host_sh_$fb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/host_sh_$fb.log').read().strip().splitlines()[-1]);print('fb $fb sharded', round(d['value']))"
done
