#!/bin/bash
# The point-to-plane bench (640x480) for the default library and each
# variant under lib/variants.   TAG=x VARIANTS="a b" bash scripts/gpu_p2plane_ab.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ppab}
for V in default ${VARIANTS}; do
  if [ "$V" = default ]; then LIBV=""; else LIBV="$PWD/realsensetracker_amd/lib/variants/$V.so"; fi
  RST_LIB=$LIBV timeout -k 10 300 python bench.py --mode p2plane --no-host-api --no-gicp --no-cpu ${EXTRA:-} > gpurun_out/${TAG}_${V}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${V}.log; exit 1; }
  grep '"metric"' gpurun_out/${TAG}_${V}.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$V value', round(d['value']), {k: round(v, 1) for k, v in d['roofline']['kernels_avg_us'].items()})"
done
