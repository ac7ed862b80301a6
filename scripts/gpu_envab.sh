#!/bin/bash
# value A/B of a runtime knob: the driver's command without the side legs,
# twice each, interleaved.  ENVB="RST_X=1" TAG=x bash scripts/gpu_envab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
TAG=${TAG:-envab}
B="--no-cpu --no-p2plane --no-gicp --ref-steps 0 --no-host-api --steps 20 --warmup 5 ${BENCH_ARGS}"
for rep in 1 2; do
  for cfg in "X=0" "${ENVB}"; do
    env $cfg timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_$rep.log 2>&1 || { tail -5 gpurun_out/${TAG}_$rep.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_$rep.log').read().strip().splitlines()[-1]);print('$cfg rep $rep value', round(d['value']), 'ok', d['pairs_ok'], {k: round(v, 1) for k, v in d['roofline'].get('kernels_avg_us', {}).items()})"
  done
done
