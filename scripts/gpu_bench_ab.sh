#!/bin/bash
# Batched value bench (and the fp64 leg) for the default library and each
# variant under lib/variants.   TAG=x VARIANTS="a b" bash scripts/gpu_bench_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-24}
TAG=${TAG:-bab}
B="--no-cpu --no-p2plane --no-gicp --no-sharded --ref-steps ${REFSTEPS:-48} --roof-steps 1 --no-host-api --batch 8 --inflight 4 --steps ${STEPS:-96}"
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  RST_LIB=$LIBV timeout -k 10 300 python bench.py $B > gpurun_out/${TAG}_${V}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${V}.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${V}.log').read().strip().splitlines()[-1]);f=d.get('fp64_sums',{});print('$V value', round(d['value']), 'fp64', round(f.get('iterations_per_s',0)), 'ok', d['pairs_ok'], {k: round(v, 1) for k, v in d['roofline']['kernels_avg_us'].items()})"
done
