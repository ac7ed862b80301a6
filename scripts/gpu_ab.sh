#!/bin/bash
# Value A/B of library variants (lib/variants/V.so): the driver's command
# without the side legs, twice each, interleaved.  TAG=x VARIANTS="a b" bash scripts/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-ab}
B="--no-cpu --no-p2plane --no-gicp --no-sharded --ref-steps 0 --no-host-api --steps 20 --warmup 5 ${BENCH_ARGS}"
for rep in 1 2; do
  for V in default ${VARIANTS}; do
    if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
    RST_LIB=$LIBV timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_${V}_$rep.log 2>&1 || { tail -5 gpurun_out/${TAG}_${V}_$rep.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${V}_$rep.log').read().strip().splitlines()[-1]);print('$V rep $rep value', round(d['value']), 'ok', d['pairs_ok'], {k: round(v, 1) for k, v in d['roofline']['kernels_avg_us'].items()})"
  done
done
