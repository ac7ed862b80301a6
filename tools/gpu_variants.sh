#!/bin/bash
# Per-iteration kernel profile (one pair in flight) of the default library
# and of each variant build given: TAG=x bash tools/gpu_variants.sh walk3 adj2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-var}
B="bench.py --inflight 1 --steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0"
for v in default "$@"; do
  if [ "$v" = default ]; then LIBV=realsensetracker_amd/lib/librst_align.so; else LIBV=realsensetracker_amd/lib/variants/$v.so; fi
  RST_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$v -o run -- python3 $B > gpurun_out/${TAG}_$v.log 2>&1 || exit $?
  echo "== $v"; grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$v.log | head -1
  python3 scripts/iter_profile.py $(find gpurun_out/${TAG}_$v -name "*kernel_trace.csv") | tee gpurun_out/${TAG}_${v}_iters.txt
done
