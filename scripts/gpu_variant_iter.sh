#!/bin/bash
# Per variant library: the stream bench and a one-pair per-iteration trace.
#   VARIANTS="a b" bash scripts/gpu_variant_iter.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# the queue count is read at the HIP runtime's first call, which rocprofv3's
# preloaded library makes before bench.py runs: set it here, not in bench.py
export GPU_MAX_HW_QUEUES=24
for v in default ${VARIANTS}; do
  lib=$PWD/realsensetracker_amd/lib/librst_align.so
  [ "$v" != default ] && lib=$PWD/realsensetracker_amd/lib/variants/$v.so
  f=gpurun_out/vi_${v}.log
  RST_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 > $f 2>&1 || exit $?
  echo "$v: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps", d["roofline"]["kernels_avg_us"])')"
  RST_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/vit_${v} -o run -- python3 bench.py --inflight 1 --steps 6 --warmup 1 --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 > gpurun_out/vit_${v}.log 2>&1 || exit $?
  python3 scripts/iter_profile.py $(find gpurun_out/vit_${v} -name "*kernel_trace.csv") | tail -14
done
