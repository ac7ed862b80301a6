#!/bin/bash
# run-time knobs of the value leg (env / bench flags), default library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--no-cpu --no-p2plane --no-gicp --no-sharded --ref-steps 0 --no-host-api --steps 20 --warmup 5"
run() {  # name, env..., -- , args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py $B $EXTRA > gpurun_out/env_$name.log 2>&1 || { tail -3 gpurun_out/env_$name.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/env_$name.log').read().strip().splitlines()[-1]);print('$name value', round(d['value']), 'ok', d['pairs_ok'])"
}
export GPU_MAX_HW_QUEUES=24
run base X=1
run fb256 RST_FB_BLOCKS=256
run fb512 RST_FB_BLOCKS=512
run fb768 RST_FB_BLOCKS=768
run lmf8k RST_LANE_MIN_FLOOR=8192
run lmf32k RST_LANE_MIN_FLOOR=32768
EXTRA="--prep-threads 2" run prep2 X=1
EXTRA="--prep-threads 4" run prep4 X=1
EXTRA="--hw-queues 16" run hwq16 X=1
EXTRA="--hw-queues 32" run hwq32 X=1
run base2 X=1
