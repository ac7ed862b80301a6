#!/bin/bash
# Stream bench under run-time knobs (environment), e.g.
#   ENVS="RST_FB_BLOCKS=512 RST_FB_BLOCKS=2048" bash scripts/gpu_env_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for e in "" ${ENVS}; do
  f=gpurun_out/envsweep_${e:-default}.log
  env $e timeout -k 10 300 python bench.py --no-cpu --no-p2plane --no-host-api --no-gicp --ref-steps 0 > $f 2>&1 || exit $?
  echo "${e:-default}: $(grep '^{' $f | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"]), "it/s", round(d["frames_per_s"],1), "fps")')"
done
